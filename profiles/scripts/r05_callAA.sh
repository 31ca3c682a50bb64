#!/bin/bash
# Round 5 call AA: config 5 at HEAD with the user pass's sources queued largest first (the
# default now) against id order (BLP_LPT=0): one sharded bench line each, parity included.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
c5() {  # name, env...
  local n=$1
  shift
  env "$@" timeout -k 10 900 python -u bench.py --mode sharded --config c5 --steps 3 --warmup 1 > gpurun_out/r05aa_$n.json 2> gpurun_out/r05aa_$n.err || { tail -20 gpurun_out/r05aa_$n.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r05aa_$n.json').read().strip().splitlines()[-1]);print('$n', round(d['ms_per_step'],3), d['value'], d.get('parity'), d.get('kernels_ms'), d.get('setup_s'))"
}
c5 def
c5 idorder BLP_LPT=0
