#!/bin/bash
# Round 3: pipelined k_score_split variants (BLP_SPLIT_XP bits: 1 = short-slice partials via LDS
# and the output half, 2 = no row prefetch) on the config-5 user pass.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
q() {  # name, args...
  local n=$1; shift
  timeout -k 10 900 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/e24_$n.json 2> gpurun_out/e24_$n.err || { tail -20 gpurun_out/e24_$n.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/e24_$n.json'));print('$n', round(d['ms_per_step'],3), d['roofline'].get('kernel_ms'), d.get('parity',{}).get('ok'))"
}
for xp in 0 1 2 3; do
  BLP_SPLIT_XP=$xp q user_xp$xp --mode sharded --config c5 --steps 3 --warmup 1 --no-parity --sides user || exit 1
done
