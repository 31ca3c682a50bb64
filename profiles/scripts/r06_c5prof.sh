#!/bin/bash
# Round 6: config-5 kernel traces, one per pass (--sides user / business, 2 timed steps each), so
# that no kernel's duration includes waiting for the other pass's persistent grid.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for side in business user; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06c5prof_$side -o c5 -- python3 bench.py --mode sharded --config c5 --sides $side --steps 2 --warmup 1 --no-parity --no-cpu-baseline > gpurun_out/r06c5prof_$side.json 2> gpurun_out/r06c5prof_$side.err || { tail -20 gpurun_out/r06c5prof_$side.err; exit 1; }
  PROFILE_OUT=gpurun_out python3 profiles/summarize.py r06_c5prof_$side $(find gpurun_out/r06c5prof_$side -name "*.db") > /dev/null || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/r06c5prof_$side.json').read().strip().splitlines()[-1]);print('$side', round(d['ms_per_step'],2))"
  head -14 gpurun_out/r06_c5prof_$side.md | cut -c1-160
done
