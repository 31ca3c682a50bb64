#!/bin/bash
# Round 5: HIP API + memory-copy + kernel timeline of one config-2 similarity.main run (no
# counters), to see what the 20-40 ms synchronous copies wait on. CSV under gpurun_out/r05_e2e_trace.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
P=/tmp/prof_e2e
rm -rf $P
cd /tmp && export TMPDIR=/tmp
BLP_SLOW_HIP_MS=3 timeout -s KILL 300 rocprofv3 --hip-trace --memory-copy-trace --kernel-trace --output-format csv -d $P -o e2e -- python3 $R/bench.py --mode e2e --config c2 > $R/gpurun_out/r05_e2e_trace.json 2> $R/gpurun_out/r05_e2e_trace.err || exit 1
mkdir -p $R/gpurun_out/r05_e2e_trace
for f in $(find $P -name "*.csv"); do gzip -c $f > $R/gpurun_out/r05_e2e_trace/$(basename $f).gz; done
ls -la $R/gpurun_out/r05_e2e_trace
