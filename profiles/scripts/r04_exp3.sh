#!/bin/bash
# Round 4, experiment 3: does the large scorer's per-segment synchronisation matter? Config-2
# user side alone with 512-pair scan segments (HEAD) against 256 (libblp_exp_seg256.so), alternating.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
q() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --sides user --no-cpu-baseline --no-exchange --steps 20 --warmup 3 > gpurun_out/e3_$name.json 2> gpurun_out/e3_$name.err || { tail -5 gpurun_out/e3_$name.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/e3_$name.json'));print('$name', round(d['ms_per_step'],4), round(d['kernels_ms']['user']['score_ms'],4))"
}
L=$R/bipartite-link-prediction_amd/blp/libblp_exp_seg256.so
q seg512a BLP_X=0 && q seg256a BLP_LIB=$L && q seg512b BLP_X=0 && q seg256b BLP_LIB=$L
