#!/bin/bash
# Round 3: config-3 top-k after the dense hot-target counts -- phase clocks (BLP_PROF build) and
# the hot-set threshold / per-source cap.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
BLP_LIB=$R/bipartite-link-prediction_amd/blp/libblp_tkprof.so timeout -k 10 300 python profiles/scripts/topk_probe.py || exit 1
BLP_TOPK_NO_DENSE=1 BLP_LIB=$R/bipartite-link-prediction_amd/blp/libblp_tkprof.so timeout -k 10 300 python profiles/scripts/topk_probe.py || exit 1
q() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/e14_$n.json 2> gpurun_out/e14_$n.err || { tail -20 gpurun_out/e14_$n.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/e14_$n.json'));print('$n', round(d['ms_per_step'],3), d.get('work'))"
}
BLP_TOPK_DENSE_F=3 q f3 --mode topk --steps 5 --warmup 1 --no-parity || exit 1
BLP_TOPK_DENSE_F=5 q f5 --mode topk --steps 5 --warmup 1 --no-parity || exit 1
BLP_TOPK_DENSE_F=8 q f8 --mode topk --steps 5 --warmup 1 --no-parity || exit 1
BLP_TOPK_DENSE_MAX=3 q m3 --mode topk --steps 5 --warmup 1 --no-parity || exit 1
