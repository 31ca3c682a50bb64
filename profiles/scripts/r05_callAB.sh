#!/bin/bash
# Round 5 call AB: the top-k claim order's work estimate -- wedges, sum |N(b)| (default, 1) against
# pushes, sum w2[b] plus the dense adds' words (2) and list order (0): the top-k tests, then
# config-3 bench lines alternating.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_topk.py > gpurun_out/r05ab_tests.log 2>&1 || { tail -30 gpurun_out/r05ab_tests.log; exit 1; }
tail -2 gpurun_out/r05ab_tests.log
tk() {  # name, env...
  local n=$1
  shift
  env "$@" timeout -k 10 300 python bench.py --mode topk --steps 10 > gpurun_out/r05ab_$n.json 2> gpurun_out/r05ab_$n.err || { tail gpurun_out/r05ab_$n.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r05ab_$n.json').read().strip().splitlines()[-1]);print('$n', d['ms_per_step'], d.get('parity', {}).get('jaccard_exact'))"
}
for i in 1 2 3; do
  tk o1_$i
  tk o2_$i BLP_TK_ORDER=2
done
tk o0_1 BLP_TK_ORDER=0
