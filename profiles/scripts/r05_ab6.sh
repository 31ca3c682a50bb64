#!/bin/bash
# Round 5 A/B 6: config 3 -- top-k selection rounds with one barrier (default) against two
# (libblp_exp4.so, -DBLP_TK_ONEBAR=0), top-k tests first; then the config-5 profile at HEAD
# (trace + FETCH/WRITE + SQ/TCC of both passes, r05_c5).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_topk.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05ab6_tests.log 2>&1 || { tail -60 gpurun_out/r05ab6_tests.log; exit 1; }
tail -1 gpurun_out/r05ab6_tests.log
tk() {  # name, env...
  local n=$1
  shift
  env "$@" timeout -k 10 600 python bench.py --mode topk --no-cpu-baseline > gpurun_out/r05ab6_$n.json 2> gpurun_out/r05ab6_$n.err || { tail -20 gpurun_out/r05ab6_$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r05ab6_$n.json'));print('$n', round(d['ms_per_step'],3), d['value'], d.get('parity'))"
}
for i in 1 2; do
  tk one_$i
  tk two_$i BLP_LIB=$R/bipartite-link-prediction_amd/blp/libblp_exp4.so
done
bash profiles/scripts/r05_prof.sh r05_c5 600 --mode sharded --config c5 --steps 3 || exit 1
