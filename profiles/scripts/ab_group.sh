#!/bin/bash
# A/B of the bucket-sort grouping (business pass): HEAD library (libblp_prev.so) against the
# working tree (libblp.so), config 2, each twice, interleaved; then the business pass alone.
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_similarity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_group_tests.log 2>&1 || { tail -30 gpurun_out/ab_group_tests.log; exit 1; }
tail -1 gpurun_out/ab_group_tests.log
run() {  # name, lib, extra args
  BLP_LIB=$PWD/bipartite-link-prediction_amd/blp/$2 timeout -k 10 300 python bench.py --no-cpu-baseline "${@:3}" \
    > gpurun_out/ab_$1.json 2> gpurun_out/ab_$1.err || { tail -30 gpurun_out/ab_$1.err; exit 1; }
  python - "$1" <<'EOF'
import json, sys
d = json.loads(open(f"gpurun_out/ab_{sys.argv[1]}.json").read().strip().splitlines()[-1])
print(sys.argv[1], d["ms_per_step"], d.get("kernels_ms"), flush=True)
EOF
}
run prev1 libblp_prev.so && run new1 libblp.so && run prev2 libblp_prev.so && run new2 libblp.so &&
  run prevbus libblp_prev.so --sides business && run newbus libblp.so --sides business
