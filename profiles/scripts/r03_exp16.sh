#!/bin/bash
# Round 3: top-k dense counts with dense AA words in the hash / direct passes -- tests (bound-
# checked and release), then the hot-set threshold x per-source cap sweep at config 3.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
L=$R/bipartite-link-prediction_amd/blp
BLP_LIB=$L/libblp_debug.so timeout -k 10 300 python -u -m pytest tests/test_gpu_topk.py -x -q --timeout 120 --timeout-method thread > gpurun_out/e16_topk_debug.log 2>&1 || { tail -30 gpurun_out/e16_topk_debug.log; exit 1; }
tail -2 gpurun_out/e16_topk_debug.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_topk.py -x -q --timeout 120 --timeout-method thread > gpurun_out/e16_topk.log 2>&1 || { tail -30 gpurun_out/e16_topk.log; exit 1; }
tail -2 gpurun_out/e16_topk.log
q() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/e16_$n.json 2> gpurun_out/e16_$n.err || { tail -20 gpurun_out/e16_$n.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/e16_$n.json'));w=d.get('work');print('$n', round(d['ms_per_step'],3), w['pushed'], w['dense_target_adds'], d.get('parity'))"
}
q def --mode topk --steps 5 --warmup 1 || exit 1
for f in 8 12 16 24; do
  for m in 3 4 8; do
    BLP_TOPK_DENSE_F=$f BLP_TOPK_DENSE_MAX=$m q f${f}_m$m --mode topk --steps 5 --warmup 1 --no-parity || exit 1
  done
done
