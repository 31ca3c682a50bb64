#!/bin/bash
# Round 3: config 5 per pass (user side alone, business side alone, both) with XCD-grouped split
# queues, then the config-5 profile (trace + FETCH/WRITE + SQ/TCC) of the default two-pass step.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
q() {  # name, args...
  local n=$1; shift
  timeout -k 10 400 python bench.py --no-cpu-baseline "$@" > gpurun_out/e5_$n.json 2> gpurun_out/e5_$n.err || { tail -20 gpurun_out/e5_$n.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/e5_$n.json'));print('$n', round(d['ms_per_step'],3), d['roofline'].get('kernel_ms'))"
}
q c5_user --mode sharded --config c5 --steps 3 --warmup 1 --no-parity --sides user || exit 1
q c5_both --mode sharded --config c5 --steps 3 --warmup 1 --no-parity || exit 1
bash profiles/scripts/r03_prof.sh r03_c5_v2 --mode sharded --config c5 --steps 2 > gpurun_out/e5_prof.log 2>&1 || { tail -20 gpurun_out/e5_prof.log; exit 1; }
grep -B1 -A18 "k_score_split" gpurun_out/r03_c5_v2_pmc.txt | head -42
