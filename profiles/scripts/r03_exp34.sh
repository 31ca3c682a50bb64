#!/bin/bash
# Round 3: hash-routed business sources on two table sizes (small: 16 KiB tables, 256 threads,
# 8 workgroups per CU; large: as before) behind a 3-way partition of the active list -- GPU tests
# of the split / hash paths, config 5 with parity, the business pass alone (and its kernel trace),
# the user pass alone in chunk-major item order (BLP_SPLIT_ONEQ=2) and in the default order.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_similarity.py tests/test_gpu_ingest.py > gpurun_out/e34_tests.log 2>&1 || { tail -30 gpurun_out/e34_tests.log; exit 1; }
tail -2 gpurun_out/e34_tests.log
q() {  # name, args...
  local n=$1; shift
  timeout -k 10 600 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/e34_$n.json 2> gpurun_out/e34_$n.err || { tail -20 gpurun_out/e34_$n.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/e34_$n.json'));print('$n', round(d['ms_per_step'],3), d['roofline'].get('kernel_ms'), d.get('parity',{}).get('ok'))"
}
q c5 --mode sharded --config c5 --steps 3 --warmup 1 || exit 1
q bus --mode sharded --config c5 --steps 3 --warmup 1 --no-parity --sides business || exit 1
BLP_SPLIT_ONEQ=2 q user_cmajor --mode sharded --config c5 --steps 3 --warmup 1 --no-parity --sides user || exit 1
q user --mode sharded --config c5 --steps 3 --warmup 1 --no-parity --sides user || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 400 rocprofv3 --kernel-trace --stats -d /tmp/p34 -o bus -- python3 $R/bench.py --mode sharded --config c5 --steps 3 --warmup 1 --no-parity --no-cpu-baseline --sides business > $R/gpurun_out/e34_prof.log 2>&1 || { tail -20 $R/gpurun_out/e34_prof.log; exit 1; }
f=$(find /tmp/p34 -name "*kernel_stats.csv" | head -1)
cp $f $R/gpurun_out/r03_c5_business_v3_kernel_stats.csv
head -12 $f | cut -c1-220
