#!/bin/bash
# Round 3: the hash-set routing bound re-measured after the partition and the 4-source claims:
# config-5 business pass alone at BLP_HASH_WORK = default (8192), 12000, 5000.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
q() {  # name, args...
  local n=$1; shift
  timeout -k 10 600 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/e37_$n.json 2> gpurun_out/e37_$n.err || { tail -20 gpurun_out/e37_$n.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/e37_$n.json'));print('$n', round(d['ms_per_step'],3), d['roofline'].get('kernel_ms'))"
}
B="--mode sharded --config c5 --steps 3 --warmup 1 --no-parity --sides business"
q bus_8k $B || exit 1
BLP_HASH_WORK=12000 q bus_12k $B || exit 1
BLP_HASH_WORK=5000 q bus_5k $B || exit 1
grep -h "plan business" gpurun_out/e37_*.err
