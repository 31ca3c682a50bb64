#!/bin/bash
# Round 3: dense counts of hot targets in the top-k count pass -- top-k tests under the bound-
# checked build and the release build, then config 3 with and without (BLP_TOPK_NO_DENSE=1),
# and the similarity tests (item grouping with staged records).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
L=$R/bipartite-link-prediction_amd/blp
BLP_LIB=$L/libblp_debug.so timeout -k 10 300 python -u -m pytest tests/test_gpu_topk.py -x -q --timeout 120 --timeout-method thread > gpurun_out/e12_topk_debug.log 2>&1 || { tail -30 gpurun_out/e12_topk_debug.log; exit 1; }
tail -2 gpurun_out/e12_topk_debug.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_topk.py -x -q --timeout 120 --timeout-method thread > gpurun_out/e12_topk.log 2>&1 || { tail -30 gpurun_out/e12_topk.log; exit 1; }
tail -2 gpurun_out/e12_topk.log
q() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/e12_$n.json 2> gpurun_out/e12_$n.err || { tail -20 gpurun_out/e12_$n.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/e12_$n.json'));print('$n', round(d['ms_per_step'],3), d['roofline'].get('kernel_ms'), d.get('work'), d.get('parity'))"
}
q topk --mode topk --steps 5 --warmup 1 || exit 1
BLP_TOPK_NO_DENSE=1 q topk_nodense --mode topk --steps 5 --warmup 1 --no-parity || exit 1
BLP_TOPK_DENSE_F=1 q topk_f1 --mode topk --steps 5 --warmup 1 --no-parity || exit 1
BLP_TOPK_DENSE_MAX=16 q topk_m16 --mode topk --steps 5 --warmup 1 --no-parity || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_similarity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/e12_sim.log 2>&1 || { tail -30 gpurun_out/e12_sim.log; exit 1; }
tail -2 gpurun_out/e12_sim.log
