#!/bin/bash
# Round 3: split scorer with the short-slice metadata loaded ahead (split entries of g + NW and
# y of g + 2 NW in flight while group g's row is tested) -- GPU tests of the split paths, config 5
# with parity (both sides), the user pass alone, the business pass alone (hash sources now
# partitioned to the front of the active list).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_similarity.py tests/test_gpu_ingest.py tests/test_gpu_headline.py > gpurun_out/e32_tests.log 2>&1 || { tail -30 gpurun_out/e32_tests.log; exit 1; }
tail -2 gpurun_out/e32_tests.log
q() {  # name, args...
  local n=$1; shift
  timeout -k 10 900 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/e32_$n.json 2> gpurun_out/e32_$n.err || { tail -20 gpurun_out/e32_$n.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/e32_$n.json'));print('$n', round(d['ms_per_step'],3), d['roofline'].get('kernel_ms'), d.get('parity',{}).get('ok'))"
}
q c5 --mode sharded --config c5 --steps 3 --warmup 1 || exit 1
q c5_user --mode sharded --config c5 --steps 3 --warmup 1 --no-parity --sides user || exit 1
q c5_bus --mode sharded --config c5 --steps 3 --warmup 1 --no-parity --sides business || exit 1
grep -h "plan " gpurun_out/e32_*.err
