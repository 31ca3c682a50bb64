#!/bin/bash
# Round 3: k_score_split with wave-independent short slices (no block barrier inside a round of
# 4 groups per wave) and the long slices queued per round -- GPU tests, then the config-5 user
# pass against the committed kernel (libblp_old.so), then config 5 with parity.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_similarity.py tests/test_gpu_ingest.py tests/test_gpu_headline.py > gpurun_out/e29_tests.log 2>&1 || { tail -30 gpurun_out/e29_tests.log; exit 1; }
tail -2 gpurun_out/e29_tests.log
q() {  # name, args...
  local n=$1; shift
  timeout -k 10 900 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/e29_$n.json 2> gpurun_out/e29_$n.err || { tail -20 gpurun_out/e29_$n.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/e29_$n.json'));print('$n', round(d['ms_per_step'],3), d['roofline'].get('kernel_ms'), d.get('parity',{}).get('ok'))"
}
q user_new --mode sharded --config c5 --steps 3 --warmup 1 --no-parity --sides user || exit 1
BLP_LIB=$R/bipartite-link-prediction_amd/blp/libblp_old.so q user_old --mode sharded --config c5 --steps 3 --warmup 1 --no-parity --sides user || exit 1
q c5 --mode sharded --config c5 --steps 3 --warmup 1 || exit 1
