#!/bin/bash
# Round 6, A/B 12, alternating on one box: config 2, the user scorer's row-chunk scan reading the
# code weights of all K ids with the bitmap words (libblp.so, HEAD) against reading them after the
# hit mask, with every non-hit id reading entry 0 (a broadcast: fewer bank conflicts, one more
# dependent LDS round trip; libblp_wt.so, -DBLP_WT_AFTER=1). The first wt arm checks parity.
# Result (r06_ab12.txt): 1.731-1.738 against 1.719-1.725 ms, slower; the macro was removed.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
L=$R/bipartite-link-prediction_amd/blp
run() {  # name lib extra
  BLP_LIB=$L/$2 timeout -k 10 300 python bench.py --no-cpu-baseline --no-exchange $3 > gpurun_out/r06ab12_$1.json 2> gpurun_out/r06ab12_$1.err || { tail -20 gpurun_out/r06ab12_$1.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r06ab12_$1.json'));print('$1', round(d['ms_per_step'],4), {k: {kk: round(vv, 4) for kk, vv in x.items()} for k, x in d['kernels_ms'].items()}, (d.get('parity') or {}).get('ok'))"
}
run wt_0 libblp_wt.so "" && run head_1 libblp.so --no-parity && run wt_1 libblp_wt.so --no-parity && run head_2 libblp.so --no-parity && run wt_2 libblp_wt.so --no-parity && run head_3 libblp.so --no-parity && run wt_3 libblp_wt.so --no-parity
