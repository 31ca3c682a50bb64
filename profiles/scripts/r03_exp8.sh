#!/bin/bash
# Round 3: item grouping (config 2 A/B against the bucket grouping) and the hash-set scorer for light split-batch sources -- similarity tests under the bound-checked
# build and the release build, then config 5 with and without it (both sides, business side alone).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
L=$R/bipartite-link-prediction_amd/blp
BLP_LIB=$L/libblp_debug.so timeout -k 10 400 python -u -m pytest tests/test_gpu_similarity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/e8_sim_debug.log 2>&1 || { tail -30 gpurun_out/e8_sim_debug.log; exit 1; }
tail -2 gpurun_out/e8_sim_debug.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_similarity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/e8_sim.log 2>&1 || { tail -30 gpurun_out/e8_sim.log; exit 1; }
tail -2 gpurun_out/e8_sim.log
q() {  # name, args...
  local n=$1; shift
  timeout -k 10 900 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/e8_$n.json 2> gpurun_out/e8_$n.err || { tail -20 gpurun_out/e8_$n.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/e8_$n.json'));print('$n', round(d['ms_per_step'],3), d['roofline'].get('kernel_ms'), d.get('kernels_ms'), d.get('parity'))"
}
q c2 --steps 20 --warmup 3 || exit 1
BLP_GROUP_BUCKETS=1 q c2_buckets --steps 20 --warmup 3 --no-parity || exit 1
q c5_bus --mode sharded --config c5 --steps 3 --warmup 1 --no-parity --sides business || exit 1
BLP_NO_HASH=1 q c5_bus_nohash --mode sharded --config c5 --steps 3 --warmup 1 --no-parity --sides business || exit 1
q c5 --mode sharded --config c5 --steps 3 --warmup 1 || exit 1
BLP_NO_HASH=1 q c5_nohash --mode sharded --config c5 --steps 3 --warmup 1 --no-parity || exit 1
