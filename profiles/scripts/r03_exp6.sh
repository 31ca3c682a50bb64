#!/bin/bash
# Round 3: code-ordered rows for the large scorer's Adamic-Adar scan (default) vs the id-ordered
# stream (BLP_NO_CSORT=1) on config 2, after the similarity GPU tests.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_similarity.py tests/test_gpu_headline.py -x -q --timeout 200 --timeout-method thread > gpurun_out/e6_tests.log 2>&1 || { tail -30 gpurun_out/e6_tests.log; exit 1; }
tail -2 gpurun_out/e6_tests.log
q() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/e6_$n.json 2> gpurun_out/e6_$n.err || { tail -20 gpurun_out/e6_$n.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/e6_$n.json'));print('$n', round(d['ms_per_step'],3), {k:(round(v['score_ms'],3),round(v['group_ms'],3)) for k,v in d.get('kernels_ms',{}).items()}, (d.get('parity') or {}).get('ok'), d.get('setup_s',{}).get('graph_build'))"
}
q c2 || exit 1
for r in 1 2; do
  BLP_NO_CSORT=1 q c2_nocs_$r --no-parity || exit 1
  q c2_cs_$r --no-parity || exit 1
done
q c2u --no-parity --sides user || exit 1
BLP_NO_CSORT=1 q c2u_nocs --no-parity --sides user || exit 1
