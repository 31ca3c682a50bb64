#!/bin/bash
# Round 3: wave-flattened top-k push -- the top-k tests under the BLP_DEBUG bound checks, then on the
# release build, then config 3 A/B against the row-per-lane push (libblp_x5.so, -DBLP_TK_FLAT=0).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
L=$R/bipartite-link-prediction_amd/blp
BLP_LIB=$L/libblp_debug.so timeout -k 10 300 python -u -m pytest tests/test_gpu_topk.py -x -q --timeout 120 --timeout-method thread > gpurun_out/e7_topk_debug.log 2>&1 || { tail -30 gpurun_out/e7_topk_debug.log; exit 1; }
tail -2 gpurun_out/e7_topk_debug.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_topk.py -x -q --timeout 120 --timeout-method thread > gpurun_out/e7_topk.log 2>&1 || { tail -30 gpurun_out/e7_topk.log; exit 1; }
tail -2 gpurun_out/e7_topk.log
q() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/e7_$n.json 2> gpurun_out/e7_$n.err || { tail -20 gpurun_out/e7_$n.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/e7_$n.json'));print('$n', round(d['ms_per_step'],3), d['roofline'].get('kernel_ms'), d.get('parity'))"
}
q topk --mode topk --steps 5 --warmup 1 || exit 1
BLP_LIB=$L/libblp_x5.so q topk_x5 --mode topk --steps 5 --warmup 1 --no-parity || exit 1
q topk_b --mode topk --steps 5 --warmup 1 --no-parity || exit 1
