#!/bin/bash
# Round 3: config 5 with both passes as one co-scheduled step (chunk-parallel grids on CU shares
# in proportion to their planned work) vs the passes one after the other; share sweep.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
q() {  # name, args...
  local n=$1; shift
  timeout -k 10 900 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/e17_$n.json 2> gpurun_out/e17_$n.err || { tail -20 gpurun_out/e17_$n.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/e17_$n.json'));print('$n', round(d['ms_per_step'],3), d['roofline'].get('kernel_ms'), d.get('parity'))"
}
q c5_cosched --mode sharded --config c5 --steps 3 --warmup 1 --no-parity || exit 1
q c5_serial --mode sharded --config c5 --steps 3 --warmup 1 --no-parity --serial-passes || exit 1
BLP_SPLIT_COSCHED_CUS=176 q c5_u176 --mode sharded --config c5 --steps 3 --warmup 1 --no-parity || exit 1
BLP_SPLIT_COSCHED_CUS=128 q c5_u128 --mode sharded --config c5 --steps 3 --warmup 1 --no-parity || exit 1
