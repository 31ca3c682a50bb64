#!/bin/bash
# Round 3: A/B of the large scorer's fused offset scan (x2 = off) and one-word AA step sums
# (x3 = off; x4 = both off) on config 2; XCD-grouped item queues of the split scorer on config 5
# (BLP_SPLIT_ONEQ=1: one queue); the hop-3 read-before-OR kernel time; parity first.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
L=$R/bipartite-link-prediction_amd/blp
timeout -k 10 600 python -u -m pytest tests/test_gpu_similarity.py tests/test_gpu_hop3.py tests/test_gpu_headline.py -x -q --timeout 200 --timeout-method thread > gpurun_out/e4_tests.log 2>&1 || { tail -30 gpurun_out/e4_tests.log; exit 1; }
tail -2 gpurun_out/e4_tests.log
q() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/e4_$n.json 2> gpurun_out/e4_$n.err || { tail -20 gpurun_out/e4_$n.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/e4_$n.json'));print('$n', round(d['ms_per_step'],3), {k:(round(v['score_ms'],3),round(v['group_ms'],3)) for k,v in d.get('kernels_ms',{}).items()}, d['roofline'].get('kernel_ms'), (d.get('parity') or {}).get('ok'), d.get('setup_s',{}).get('hop3_kernel_ms'))"
}
q c2 || exit 1
for r in 1 2; do
  for v in x2 x3 x4; do BLP_LIB=$L/libblp_$v.so q c2_${v}_$r --no-parity || exit 1; done
  q c2_d_$r --no-parity || exit 1
done
q c5 --mode sharded --config c5 --steps 3 --warmup 1 --no-parity || exit 1
BLP_SPLIT_ONEQ=1 q c5_oneq --mode sharded --config c5 --steps 3 --warmup 1 --no-parity || exit 1
