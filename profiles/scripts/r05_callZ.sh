#!/bin/bash
# Round 5 call Z: which pass of a pair takes the highest-priority stream (BLP_PAIR_HI_SECOND=1: the
# business pass), with and without the user pass queued largest first (BLP_LPT=1); config-2 bench
# lines alternating.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
b() {  # name, env...
  local n=$1
  shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r05z_$n.json 2> gpurun_out/r05z_$n.err || { tail -20 gpurun_out/r05z_$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r05z_$n.json'));print('$n', round(d['ms_per_step'],3), {k:{kk:round(vv,3) for kk,vv in v.items()} for k,v in d['kernels_ms'].items()}, d['parity']['ok'], d.get('including_batch_create'))"
}
for i in 1 2 3; do
  b def_$i
  b lpt_$i BLP_LPT=1
  b hi2_$i BLP_PAIR_HI_SECOND=1
  b lpt_hi2_$i BLP_LPT=1 BLP_PAIR_HI_SECOND=1
done
