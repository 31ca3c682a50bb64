#!/bin/bash
# Round 6, A/B 13, alternating on one box: config 2 with the graph-level score / group timers
# recorded beside the batch timers (default: 4 timing events per stream boundary) against the
# batch timers alone (BLP_NO_GTIMERS=1: 2 per boundary). The kernel trace (r06_c2trace) shows a
# ~20 us idle gap on the user stream at each boundary that has only event records in it.
# (The experiment knob was replaced by r06_ab14's change: the graph totals from the batch timers.)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
run() {  # name env
  env $2 timeout -k 10 300 python bench.py --no-cpu-baseline --no-exchange --no-parity > gpurun_out/r06ab13_$1.json 2> gpurun_out/r06ab13_$1.err || { tail -20 gpurun_out/r06ab13_$1.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r06ab13_$1.json'));print('$1', round(d['ms_per_step'],4), {k: {kk: round(vv, 4) for kk, vv in x.items()} for k, x in d['kernels_ms'].items()})"
}
for round in 1 2 3 4; do
  run def_$round BLP_X=0 && run nogt_$round BLP_NO_GTIMERS=1 || exit 1
done
