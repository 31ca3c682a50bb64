#!/bin/bash
# Round 3: config-2 dense-row threshold sweep (rows OR-ed as bitmaps into the user-side H2).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
q() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/e19_$n.json 2> gpurun_out/e19_$n.err || { tail -20 gpurun_out/e19_$n.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/e19_$n.json'));print('$n', round(d['ms_per_step'],3), d.get('kernels_ms'), d.get('work', {}).get('user'))"
}
q d64 --steps 20 --warmup 3 --no-parity || exit 1
BLP_HOT_DENSITY=128 q d128 --steps 20 --warmup 3 --no-parity || exit 1
BLP_HOT_DENSITY=256 q d256 --steps 20 --warmup 3 --no-parity || exit 1
BLP_HOT_DENSITY=32 q d32 --steps 20 --warmup 3 --no-parity || exit 1
BLP_HOT_DENSITY=128 q d128_user --steps 20 --warmup 3 --no-parity --sides user || exit 1
q d64_user --steps 20 --warmup 3 --no-parity --sides user || exit 1
