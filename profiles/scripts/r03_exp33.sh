#!/bin/bash
# Round 3: same-box A/B of the split scorer's short-slice metadata prefetch (libblp_pf.so)
# against the plain loop (libblp.so, both with the hash/split partition of the active list):
# config-5 user pass alone, alternating, then config 5 with parity on libblp.so.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
L=$R/bipartite-link-prediction_amd/blp
q() {  # name, lib, args...
  local n=$1 lib=$2; shift 2
  BLP_LIB=$L/$lib timeout -k 10 600 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/e33_$n.json 2> gpurun_out/e33_$n.err || { tail -20 gpurun_out/e33_$n.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/e33_$n.json'));print('$n', round(d['ms_per_step'],3), d['roofline'].get('kernel_ms'), d.get('parity',{}).get('ok'))"
}
U="--mode sharded --config c5 --steps 3 --warmup 1 --no-parity --sides user"
q u_base1 libblp.so $U || exit 1
q u_pf1 libblp_pf.so $U || exit 1
q u_base2 libblp.so $U || exit 1
q u_pf2 libblp_pf.so $U || exit 1
q c5 libblp.so --mode sharded --config c5 --steps 3 --warmup 1 || exit 1
