#!/bin/bash
# Round 4, check 13: run-grouped pairs scored without grouped metadata (k_score reads y and
# N(y) bounds itself; the run pass writes no per-pair arrays) -- scorer tests, then an
# alternating A/B against the previous build (libblp_exp_prev.so).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_similarity.py tests/test_gpu_headline.py tests/test_gpu_debug.py tests/test_gpu_hop3.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04c12_gputest.log 2>&1 || { tail -60 gpurun_out/r04c12_gputest.log; exit 1; }
tail -1 gpurun_out/r04c12_gputest.log
ab() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --no-exchange --steps 20 --warmup 3 > gpurun_out/ab13_$name.json 2> gpurun_out/ab13_$name.err || { tail -5 gpurun_out/ab13_$name.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab13_$name.json'));print('$name', round(d['ms_per_step'],4), {k: round(v['score_ms'],3) for k,v in d['kernels_ms'].items()}, d.get('parity',{}).get('ok'))"
}
P=$R/bipartite-link-prediction_amd/blp/libblp_exp_prev.so
ab new1 BLP_X=0 && ab prev1 BLP_LIB=$P && ab new2 BLP_X=0 && ab prev2 BLP_LIB=$P && ab new3 BLP_X=0 && ab prev3 BLP_LIB=$P || exit 1
