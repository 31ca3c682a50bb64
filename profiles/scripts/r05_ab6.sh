#!/bin/bash
# Round 5 A/B 6: config 3 -- top-k selection rounds with one barrier (default) against two
# (libblp_exp4.so, -DBLP_TK_ONEBAR=0), top-k tests first; config 5 -- the 16-bit split table
# (default, with 50 + 50 sources' parity) against the int32 table (BLP_SPLIT32=1).
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
c5() {  # name, extra args, env...
  local n=$1 x=$2
  shift 2
  env "$@" timeout -k 10 600 python -u bench.py --mode sharded --config c5 --no-cpu-baseline $x > gpurun_out/r05ab6_$n.json 2> gpurun_out/r05ab6_$n.err || { tail -20 gpurun_out/r05ab6_$n.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r05ab6_$n.json').read().strip().splitlines()[-1]);print('$n', round(d['ms_per_step'],3), d['value'], d.get('kernels_ms'), d.get('parity',{}).get('ok'))"
}
c5 c5_s16 ""
c5 c5_s32 --no-parity BLP_SPLIT32=1
