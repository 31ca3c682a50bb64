#!/bin/bash
# Round 6, A/B 7, alternating on one box: the wedge-set launch's resident blocks per CU
# (BLP_WSET_BPC: 8 = the default; fewer blocks keep fewer users' sets in an XCD's L2 at once).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
for round in 1 2; do
  for v in 8 6 4 3 2; do
    BLP_WSET_BPC=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-exchange --no-parity > gpurun_out/r06ab7_${v}_$round.json 2> gpurun_out/r06ab7_${v}_$round.err || { tail -20 gpurun_out/r06ab7_${v}_$round.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r06ab7_${v}_$round.json'));print('bpc $v', $round, round(d['ms_per_step'],4), {k: {kk: round(vv, 4) for kk, vv in x.items()} for k, x in d['kernels_ms'].items()})"
  done
done
