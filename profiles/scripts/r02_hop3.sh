#!/bin/bash
# Hop-3 wedge-row path: its GPU tests, then a kernel trace + FETCH/WRITE passes of the default
# bench (whose example generation runs blp_hop3_sample over 10K users) -> gpurun_out/$1.{json,md}
set -o pipefail
R=$GRAFT_REPO_ROOT
NAME=${1:-r02_hop3}
cd $R || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_hop3.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${NAME}_test.log 2>&1 || { tail -30 gpurun_out/${NAME}_test.log; exit 1; }
tail -2 gpurun_out/${NAME}_test.log
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-parity"
for p in trace fetch write; do rm -rf $R/gpurun_out/prof_$p; done
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_trace -o trace -- python3 $R/bench.py $ARGS > $R/gpurun_out/${NAME}_trace.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/prof_fetch -o fetch -- python3 $R/bench.py $ARGS > $R/gpurun_out/${NAME}_fetch.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/prof_write -o write -- python3 $R/bench.py $ARGS > $R/gpurun_out/${NAME}_write.log 2>&1 || exit 1
PROFILE_OUT=$R/gpurun_out python3 $R/profiles/summarize.py $NAME $(find $R/gpurun_out/prof_trace -name "*.db") $(find $R/gpurun_out/prof_fetch -name "*.db") $(find $R/gpurun_out/prof_write -name "*.db") > /dev/null || exit 1
head -12 $R/gpurun_out/$NAME.md
grep examples $R/gpurun_out/${NAME}_trace.log
