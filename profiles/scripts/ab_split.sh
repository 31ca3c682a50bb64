#!/bin/bash
# A/B of the chunk-parallel scorer (config 4 similarity step, then config 5): HEAD library
# (libblp_prev.so) against the working tree.
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_similarity.py tests/test_gpu_ingest.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_split_tests.log 2>&1 || { tail -30 gpurun_out/ab_split_tests.log; exit 1; }
tail -1 gpurun_out/ab_split_tests.log
run() {
  BLP_LIB=$PWD/bipartite-link-prediction_amd/blp/$2 timeout -k 10 600 python bench.py --no-cpu-baseline "${@:3}" \
    > gpurun_out/abs_$1.json 2> gpurun_out/abs_$1.err || { tail -30 gpurun_out/abs_$1.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step'],3), d.get('kernels_ms'))" gpurun_out/abs_$1.json $1
}
run c4prev1 libblp_prev.so --config c4 --no-parity && run c4new1 libblp.so --config c4 --no-parity &&
run c4prev2 libblp_prev.so --config c4 --no-parity && run c4new2 libblp.so --config c4 --no-parity &&
run c5prev libblp_prev.so --mode sharded --config c5 --steps 5 --warmup 1 && run c5new libblp.so --mode sharded --config c5 --steps 5 --warmup 1
