#!/bin/bash
# Round 3: wave-contiguous row-chunk loops (BLP_RCW, default) -- GPU parity of every scorer path,
# then A/B against the block-interleaved loops (libblp_x0.so, -DBLP_RCW=0) on configs 2 and 5.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
L=$R/bipartite-link-prediction_amd/blp
timeout -k 10 600 python -u -m pytest tests/test_gpu_similarity.py tests/test_gpu_headline.py tests/test_gpu_ingest.py tests/test_gpu_topk.py -x -q --timeout 200 --timeout-method thread > gpurun_out/e2_tests.log 2>&1 || { tail -30 gpurun_out/e2_tests.log; exit 1; }
tail -2 gpurun_out/e2_tests.log
q() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/e2_$n.json 2> gpurun_out/e2_$n.err || { tail -20 gpurun_out/e2_$n.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/e2_$n.json'));print('$n', round(d['ms_per_step'],3), {k:(round(v['score_ms'],3),round(v['group_ms'],3)) for k,v in d.get('kernels_ms',{}).items()}, d['roofline'].get('kernel_ms'), (d.get('parity') or {}).get('ok'))"
}
q c2_rcw || exit 1
BLP_LIB=$L/libblp_x0.so q c2_x0 --no-parity || exit 1
q c2_rcw_b --no-parity || exit 1
BLP_LIB=$L/libblp_x0.so q c2_x0_b --no-parity || exit 1
q c2u_rcw --no-parity --sides user || exit 1
BLP_LIB=$L/libblp_x0.so q c2u_x0 --no-parity --sides user || exit 1
q topk --mode topk --steps 5 --warmup 1 --no-cpu-baseline || exit 1
timeout -k 10 900 python -u bench.py --mode sharded --config c5 --steps 3 --warmup 1 --no-parity > gpurun_out/e2_c5_rcw.json 2> gpurun_out/e2_c5_rcw.err || { tail -30 gpurun_out/e2_c5_rcw.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/e2_c5_rcw.json'));print('c5_rcw', d['ms_per_step'], d['roofline']['kernel_ms'])"
