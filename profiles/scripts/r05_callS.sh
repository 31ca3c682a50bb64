#!/bin/bash
# Round 5 call S: the short-row scorer's persistent grid held to part of the chip (BLP_SHORT_CUS),
# so the CUs the user scorer frees at its end go to the user pass's next grouping instead of
# queued business workgroups; crossed with the user CU share. Config-2 bench lines, alternating.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
b() {  # name, env...
  local n=$1
  shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r05s_$n.json 2> gpurun_out/r05s_$n.err || { tail -20 gpurun_out/r05s_$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r05s_$n.json'));print('$n', round(d['ms_per_step'],3), {k:{kk:round(vv,3) for kk,vv in v.items()} for k,v in d['kernels_ms'].items()}, d['parity']['ok'])"
}
for i in 1 2; do
  b def_$i
  b s64_$i BLP_SHORT_CUS=64
  b s96_$i BLP_SHORT_CUS=96
  b s128_$i BLP_SHORT_CUS=128
  b s96_c176_$i BLP_SHORT_CUS=96 BLP_COSCHED_CUS=176
  b s128_c176_$i BLP_SHORT_CUS=128 BLP_COSCHED_CUS=176
  b s64_c200_$i BLP_SHORT_CUS=64 BLP_COSCHED_CUS=200
done
