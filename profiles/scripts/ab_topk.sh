#!/bin/bash
# A/B of the top-k kernel (config 3): HEAD library (libblp_prev.so) against the working tree,
# each twice, interleaved; the top-k GPU tests on the working tree first.
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_topk.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_topk_tests.log 2>&1 || { tail -30 gpurun_out/ab_topk_tests.log; exit 1; }
tail -1 gpurun_out/ab_topk_tests.log
run() {
  BLP_LIB=$PWD/bipartite-link-prediction_amd/blp/$2 timeout -k 10 300 python bench.py --mode topk --no-cpu-baseline "${@:3}" \
    > gpurun_out/abt_$1.json 2> gpurun_out/abt_$1.err || { tail -30 gpurun_out/abt_$1.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],3), d['roofline']['kernel_ms'], d.get('parity'))" gpurun_out/abt_$1.json $1
}
run prev1 libblp_prev.so && run new1 libblp.so && run prev2 libblp_prev.so && run new2 libblp.so
