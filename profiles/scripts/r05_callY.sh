#!/bin/bash
# Round 5 call Y: the user pass queued largest work first (BLP_LPT=1) with the co-scheduled CU share
# re-swept (176 / 184 / 192 / 200 user CUs), and both passes largest first (BLP_LPT=3), against id
# order; the knob-matrix similarity tests first; config-2 bench lines alternating.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
b() {  # name, env...
  local n=$1
  shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r05y_$n.json 2> gpurun_out/r05y_$n.err || { tail -20 gpurun_out/r05y_$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r05y_$n.json'));print('$n', round(d['ms_per_step'],3), {k:{kk:round(vv,3) for kk,vv in v.items()} for k,v in d['kernels_ms'].items()}, d['parity']['ok'], d.get('including_batch_create'))"
}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_similarity.py -k "kernel_paths" > gpurun_out/r05y_tests.log 2>&1 || { tail -40 gpurun_out/r05y_tests.log; exit 1; }
tail -2 gpurun_out/r05y_tests.log
for i in 1 2; do
  b def_$i
  b lpt_$i BLP_LPT=1
  b lpt3_$i BLP_LPT=3
  b lpt184_$i BLP_LPT=1 BLP_COSCHED_CUS=184
  b lpt3_184_$i BLP_LPT=3 BLP_COSCHED_CUS=184
  b lpt176_$i BLP_LPT=1 BLP_COSCHED_CUS=176
  b lpt200_$i BLP_LPT=1 BLP_COSCHED_CUS=200
done
