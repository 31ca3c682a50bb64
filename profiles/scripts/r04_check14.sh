#!/bin/bash
# Round 4, check 14: barrier trims in the chunk-parallel and hash-set scorers (alternating claim
# slots; no closing barrier in the popcount sums) -- their tests, then config 5 (both passes)
# alternating against the previous build (libblp_exp_prev.so).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_similarity.py tests/test_gpu_debug.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04c14_gputest.log 2>&1 || { tail -60 gpurun_out/r04c14_gputest.log; exit 1; }
tail -1 gpurun_out/r04c14_gputest.log
q() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 600 python -u bench.py --no-cpu-baseline --mode sharded --config c5 --steps 3 --warmup 1 --no-parity > gpurun_out/ab14_$name.json 2> gpurun_out/ab14_$name.err || { tail -5 gpurun_out/ab14_$name.err; return 1; }
  python -c "import json;d=json.loads(open('gpurun_out/ab14_$name.json').read().strip().splitlines()[-1]);print('$name', round(d['ms_per_step'],2), d.get('kernels_ms'))"
}
P=$R/bipartite-link-prediction_amd/blp/libblp_exp_prev.so
q new1 BLP_X=0 && q prev1 BLP_LIB=$P && q new2 BLP_X=0 && q prev2 BLP_LIB=$P
