#!/bin/bash
# Round 3: k_score_split round length sweep (config-5 user pass; a first run also tried a
# next-group y prefetch: neutral, removed).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
q() {  # name, args...
  local n=$1; shift
  timeout -k 10 900 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/e30_$n.json 2> gpurun_out/e30_$n.err || { tail -20 gpurun_out/e30_$n.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/e30_$n.json'));print('$n', round(d['ms_per_step'],3), d['roofline'].get('kernel_ms'))"
}
for cfg in "8 0" "16 0" "32 0"; do
  set -- $cfg
  BLP_SPLIT_ROUND=$1 q r$1 --mode sharded --config c5 --steps 3 --warmup 1 --no-parity --sides user || exit 1
done
