#!/bin/bash
# Round 5 call X: run-grouped batches (the config-2 user pass) queue their sources largest estimated
# work first (BLP_LPT=1) against id order: the similarity tests (knob matrix includes BLP_LPT) and
# the headline test with it, then config-2 bench lines alternating.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_similarity.py > gpurun_out/r05x_tests.log 2>&1 || { tail -40 gpurun_out/r05x_tests.log; exit 1; }
tail -2 gpurun_out/r05x_tests.log
BLP_LPT=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_headline.py > gpurun_out/r05x_tests_headline.log 2>&1 || { tail -40 gpurun_out/r05x_tests_headline.log; exit 1; }
tail -2 gpurun_out/r05x_tests_headline.log
b() {  # name, env...
  local n=$1
  shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r05x_$n.json 2> gpurun_out/r05x_$n.err || { tail -20 gpurun_out/r05x_$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r05x_$n.json'));print('$n', round(d['ms_per_step'],3), {k:{kk:round(vv,3) for kk,vv in v.items()} for k,v in d['kernels_ms'].items()}, d['parity']['ok'], d.get('including_batch_create'))"
}
for i in 1 2 3; do
  b def_$i
  b lpt_$i BLP_LPT=1
done
