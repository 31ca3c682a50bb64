#!/bin/bash
# Round 4, experiment 2: config-5 user pass with the chunk partials' atomics performed in the
# XCD's L2 (workgroup scope; libblp_exp_l2atom.so, -DBLP_EXP_L2ATOM) against device scope.
# Timing only (the L2 variant is not exact when a source's chunks run on two XCDs).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
q() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-exchange --mode sharded --config c5 --steps 3 --warmup 1 --no-parity --sides user > gpurun_out/e2_$name.json 2> gpurun_out/e2_$name.err || { tail -5 gpurun_out/e2_$name.err; return 1; }
  python -c "import json;d=json.loads(open('gpurun_out/e2_$name.json').read().strip().splitlines()[-1]);print('$name', round(d['ms_per_step'],3), d.get('kernels_ms'))"
}
q base BLP_X=0 || exit 1
q l2atom BLP_LIB=$R/bipartite-link-prediction_amd/blp/libblp_exp_l2atom.so || exit 1
q base2 BLP_X=0 || exit 1
