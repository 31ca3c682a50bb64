#!/bin/bash
# Round 3: config-2 grouping kernels traced, item vs bucket grouping; config 5 business side
# alone with and without the hash-set scorer (routes in the plan log).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
bash profiles/scripts/r03_trace.sh r03_c2_items --steps 10 --warmup 2 || exit 1
BLP_GROUP_BUCKETS=1 bash profiles/scripts/r03_trace.sh r03_c2_buckets --steps 10 --warmup 2 || exit 1
q() {  # name, args...
  local n=$1; shift
  timeout -k 10 900 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/e9_$n.json 2> gpurun_out/e9_$n.err || { tail -20 gpurun_out/e9_$n.err; return 1; }
  grep "plan" gpurun_out/e9_$n.err | cut -c1-300
  python -c "import json;d=json.load(open('gpurun_out/e9_$n.json'));print('$n', round(d['ms_per_step'],3), d['roofline'].get('kernel_ms'), d.get('parity'))"
}
q c5_bus --mode sharded --config c5 --steps 3 --warmup 1 --no-parity --sides business || exit 1
BLP_NO_HASH=1 q c5_bus_nohash --mode sharded --config c5 --steps 3 --warmup 1 --no-parity --sides business || exit 1
BLP_HASH_WORK=16000 q c5_bus_hash16k --mode sharded --config c5 --steps 3 --warmup 1 --no-parity --sides business || exit 1
