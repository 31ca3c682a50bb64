#!/bin/bash
# Round 3: the graph's wedge-row bitmaps as pre-built H2 sets of long business sources --
# similarity and hop-3 tests, then config 2 with and without (BLP_NO_WBM_BATCH=1).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_similarity.py tests/test_gpu_hop3.py tests/test_gpu_headline.py -x -q --timeout 120 --timeout-method thread > gpurun_out/e18_tests.log 2>&1 || { tail -30 gpurun_out/e18_tests.log; exit 1; }
tail -2 gpurun_out/e18_tests.log
q() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/e18_$n.json 2> gpurun_out/e18_$n.err || { tail -20 gpurun_out/e18_$n.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/e18_$n.json'));print('$n', round(d['ms_per_step'],3), d.get('kernels_ms'), (d.get('parity') or {}).get('u_cn_exact'), (d.get('parity') or {}).get('b_jaccard_exact'))"
}
q c2 --steps 20 --warmup 3 || exit 1
BLP_NO_WBM_BATCH=1 q c2_nowbm --steps 20 --warmup 3 --no-parity || exit 1
q c2_bus --steps 20 --warmup 3 --no-parity --sides business || exit 1
BLP_NO_WBM_BATCH=1 q c2_bus_nowbm --steps 20 --warmup 3 --no-parity --sides business || exit 1
for c in 184 200 208; do BLP_COSCHED_CUS=$c q c2_cu$c --steps 20 --warmup 3 --no-parity || exit 1; done
