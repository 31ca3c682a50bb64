#!/bin/bash
# Round 3: kernel trace + stats of one bench command only (summarize.py -> gpurun_out/$NAME.{json,md});
# the rocprofv3 database stays in /tmp on the box.  usage: bash profiles/scripts/r03_trace.sh NAME [bench args...]
set -o pipefail
R=$GRAFT_REPO_ROOT
NAME=$1
shift
mkdir -p $R/gpurun_out
P=/tmp/trace_$NAME
rm -rf $P
mkdir -p $P
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $P -o trace -- python3 $R/bench.py --no-cpu-baseline --no-parity "$@" > $R/gpurun_out/${NAME}_trace.log 2>&1 || exit 1
PROFILE_OUT=$R/gpurun_out python3 $R/profiles/summarize.py $NAME $(find $P -name "*.db") > /dev/null || exit 1
rm -rf $P
head -24 $R/gpurun_out/$NAME.md | cut -c1-200
