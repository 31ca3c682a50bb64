#!/bin/bash
# Round 5 call N: the co-scheduled passes on dedicated (CU-masked) streams -- the similarity and
# headline tests; then the config-2 bench line with them (default) against each pass on its own
# pooled stream (BLP_CO_STREAMS=0), alternating, three each; then config-2 similarity.main twice.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_similarity.py tests/test_gpu_headline.py > gpurun_out/r05n_tests.log 2>&1 || { tail -40 gpurun_out/r05n_tests.log; exit 1; }
tail -2 gpurun_out/r05n_tests.log
b() {  # name, env...
  local n=$1
  shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r05n_$n.json 2> gpurun_out/r05n_$n.err || { tail -20 gpurun_out/r05n_$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r05n_$n.json'));print('$n', round(d['ms_per_step'],3), d['kernels_ms'], d['parity']['ok'])"
}
for i in 1 2 3; do
  b co_$i
  b own_$i BLP_CO_STREAMS=0
done
for i in 1 2; do
  timeout -k 10 300 python bench.py --mode e2e --config c2 > gpurun_out/r05n_e2e_$i.json 2> gpurun_out/r05n_e2e_$i.err || { tail -20 gpurun_out/r05n_e2e_$i.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r05n_e2e_$i.json').read().strip().splitlines()[-1]);print('e2e', round(d['e2e_s'],4), {k: round(v,4) for k,v in d['phases_s'].items()}, d['ok'])"
done
