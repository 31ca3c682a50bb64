#!/bin/bash
# Round 5 call W: config-3 top-k with sources claimed largest two-hop walk first (default) against
# list order (BLP_TK_ORDER=0): the top-k tests (release and bound-checked builds, at-size config 3),
# then bench lines alternating.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_topk.py tests/test_gpu_atsize.py -k "topk" > gpurun_out/r05w_tests.log 2>&1 || { tail -30 gpurun_out/r05w_tests.log; exit 1; }
tail -2 gpurun_out/r05w_tests.log
BLP_LIB=$R/bipartite-link-prediction_amd/blp/libblp_debug.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_topk.py > gpurun_out/r05w_tests_debug.log 2>&1 || { tail -30 gpurun_out/r05w_tests_debug.log; exit 1; }
tail -2 gpurun_out/r05w_tests_debug.log
tk() {  # name, env...
  local n=$1
  shift
  env "$@" timeout -k 10 300 python bench.py --mode topk --steps 10 > gpurun_out/r05w_$n.json 2> gpurun_out/r05w_$n.err || { tail gpurun_out/r05w_$n.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r05w_$n.json').read().strip().splitlines()[-1]);print('$n', d['ms_per_step'], d.get('parity'))"
}
for i in 1 2 3; do
  tk def_$i
  tk list_$i BLP_TK_ORDER=0
done
