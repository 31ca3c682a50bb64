#!/bin/bash
# Round 5 call O: why the config-2 step came out 3.4-3.5 ms (the two passes serialized) in the
# last two calls: the bench line at HEAD (default), without the device scratch cache
# (BLP_DEV_CACHE_MB=0) and without the bench's prewarm (BLP_BENCH_NO_PREWARM=1), alternating;
# then a kernel trace of the default (overlap of the two passes).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
b() {  # name, env...
  local n=$1
  shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity > gpurun_out/r05o_$n.json 2> gpurun_out/r05o_$n.err || { tail -20 gpurun_out/r05o_$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r05o_$n.json'));print('$n', round(d['ms_per_step'],3), d['kernels_ms'])"
}
for i in 1 2; do
  b def_$i
  b nocache_$i BLP_DEV_CACHE_MB=0
  b noprewarm_$i BLP_BENCH_NO_PREWARM=1
done
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/prof_o
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_o -o o -- python3 $R/bench.py --no-cpu-baseline --no-parity --steps 3 --warmup 1 > $R/gpurun_out/r05o_trace.log 2>&1 || exit 1
mkdir -p $R/gpurun_out/r05o_trace
for f in $(find /tmp/prof_o -name "*kernel_trace.csv"); do gzip -c $f > $R/gpurun_out/r05o_trace/$(basename $f).gz; done
ls $R/gpurun_out/r05o_trace
