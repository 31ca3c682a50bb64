#!/bin/bash
# Round 3: config-5 business pass on wedge rows -- kernel trace, and the hash-set routing bound.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
bash profiles/scripts/r03_trace.sh r03_c5_business_wedge --mode sharded --config c5 --steps 2 --warmup 1 --sides business || exit 1
q() {  # name, args...
  local n=$1; shift
  timeout -k 10 900 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/e21_$n.json 2> gpurun_out/e21_$n.err || { tail -20 gpurun_out/e21_$n.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/e21_$n.json'));print('$n', round(d['ms_per_step'],3), d['roofline'].get('kernel_ms'), d['roofline'].get('plan', {}).get('hash_sources'))"
}
BLP_NO_HASH=1 q bus_nohash --mode sharded --config c5 --steps 3 --warmup 1 --no-parity --sides business || exit 1
BLP_HASH_WORK=4096 q bus_h4k --mode sharded --config c5 --steps 3 --warmup 1 --no-parity --sides business || exit 1
