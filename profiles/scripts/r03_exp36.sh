#!/bin/bash
# Round 3: k_score_split claiming 2 items per atomic (after the hash-set scorer changes) --
# GPU tests of the split / hash paths, the config-5 user and business passes alone, config 5
# with parity, a kernel trace of the business pass.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_similarity.py tests/test_gpu_ingest.py > gpurun_out/e36_tests.log 2>&1 || { tail -30 gpurun_out/e36_tests.log; exit 1; }
tail -2 gpurun_out/e36_tests.log
q() {  # name, args...
  local n=$1; shift
  timeout -k 10 600 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/e36_$n.json 2> gpurun_out/e36_$n.err || { tail -20 gpurun_out/e36_$n.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/e36_$n.json'));print('$n', round(d['ms_per_step'],3), d['roofline'].get('kernel_ms'), d.get('parity',{}).get('ok'))"
}
q bus --mode sharded --config c5 --steps 3 --warmup 1 --no-parity --sides business || exit 1
q user --mode sharded --config c5 --steps 3 --warmup 1 --no-parity --sides user || exit 1
q c5 --mode sharded --config c5 --steps 3 --warmup 1 || exit 1
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/pb && timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d /tmp/pb -o trace -- python3 $R/bench.py --mode sharded --config c5 --steps 3 --warmup 1 --no-parity --no-cpu-baseline --sides business > $R/gpurun_out/e36_prof_bus.log 2>&1 || { tail -20 $R/gpurun_out/e36_prof_bus.log; exit 1; }
PROFILE_OUT=$R/gpurun_out python3 $R/profiles/summarize.py r03_c5_business_v5 $(find /tmp/pb -name "*.db") > /dev/null || exit 1
head -8 $R/gpurun_out/r03_c5_business_v5.md | cut -c1-200
