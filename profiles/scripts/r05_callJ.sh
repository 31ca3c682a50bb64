#!/bin/bash
# Round 5 call J: the 128 KiB hash-set scorer (BLP_HASH_BIG) -- its tests (oracle knob cases, the
# bound-checked debug build) and the device scratch cache test; then config 5: the user pass alone
# with the default routing against the big hash tables (users of <= 16K build ids), and both
# passes with the big tables (parity: 50 + 50 sources).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_similarity.py tests/test_gpu_debug.py -k "HASH_BIG or hash or cache or knobs" > gpurun_out/r05j_tests.log 2>&1 || { tail -40 gpurun_out/r05j_tests.log; exit 1; }
tail -2 gpurun_out/r05j_tests.log
c5() {  # name, args, env...
  local n=$1 args=$2
  shift 2
  env "$@" timeout -k 10 900 python -u bench.py --mode sharded --config c5 --warmup 1 --no-cpu-baseline $args > gpurun_out/r05j_$n.json 2> gpurun_out/r05j_$n.err || { tail -20 gpurun_out/r05j_$n.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r05j_$n.json').read().strip().splitlines()[-1]);print('$n', round(d['ms_per_step'],2), d.get('kernels_ms'), d.get('parity'), d['roofline'].get('plan'))"
}
c5 user_def "--steps 3 --sides user --no-parity"
c5 user_big "--steps 3 --sides user --no-parity" BLP_HASH_BIG=1
c5 both_big "--steps 3" BLP_HASH_BIG=1
