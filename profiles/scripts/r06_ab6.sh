#!/bin/bash
# Round 6, A/B 6, alternating on one box: the wedge-set launch enqueued at the step's start beside
# the user pass (default) against gated on the user pass's grouping (BLP_WSET_ORDER=1: the user
# scorer is dispatched first and the light launch fills the CUs its tail frees).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
for round in 1 2 3; do
  extra="--no-cpu-baseline --no-exchange"
  [ $round -gt 1 ] && extra="$extra --no-parity"
  for v in 0 1; do
    BLP_WSET_ORDER=$v timeout -k 10 300 python bench.py $extra > gpurun_out/r06ab6_${v}_$round.json 2> gpurun_out/r06ab6_${v}_$round.err || { tail -20 gpurun_out/r06ab6_${v}_$round.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r06ab6_${v}_$round.json'));print('order $v', $round, round(d['ms_per_step'],4), {k: {kk: round(vv, 4) for kk, vv in x.items()} for k, x in d['kernels_ms'].items()}, d.get('parity', {}).get('ok'))"
  done
done
