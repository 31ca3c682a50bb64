#!/bin/bash
# Round 3, first check: the top-k walk under the BLP_DEBUG bound checks (HEAD's loops, then the
# 16-byte row-tail variant), then the whole GPU suite on the release build (RCCL world-1
# exchange and headline-size parity included).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
L=$R/bipartite-link-prediction_amd/blp
BLP_LIB=$L/libblp_debug.so timeout -k 10 300 python -u -m pytest tests/test_gpu_topk.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r03_topk_debug.log 2>&1 || { tail -30 gpurun_out/r03_topk_debug.log; exit 1; }
tail -3 gpurun_out/r03_topk_debug.log
BLP_LIB=$L/libblp_debug_t16.so timeout -k 10 300 python -u -m pytest tests/test_gpu_topk.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r03_topk_debug_t16.log 2>&1 || { tail -30 gpurun_out/r03_topk_debug_t16.log; exit 1; }
tail -3 gpurun_out/r03_topk_debug_t16.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03_gputest.log 2>&1 || { tail -40 gpurun_out/r03_gputest.log; exit 1; }
tail -3 gpurun_out/r03_gputest.log
