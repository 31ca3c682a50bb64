#!/bin/bash
# Round 6, A/B 11, alternating on one box: config 5 (both passes), k_score_split's short slices
# tested id by id with a branch per id and the weight read through a pointer that is either the
# LDS code table or the global per-node table (libblp_prev.so = HEAD before the change: the
# compiler emitted a flat load and a full wait per hit) against branch-free phases -- all bitmap
# words, then all code weights from LDS, code-0 hits from the global table after (libblp.so).
# The first new arm checks parity.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
L=$R/bipartite-link-prediction_amd/blp
run() {  # name lib extra
  BLP_LIB=$L/$2 timeout -k 10 300 python -u bench.py --mode sharded --config c5 --steps 3 --warmup 1 --no-cpu-baseline $3 > gpurun_out/r06ab11_$1.json 2> gpurun_out/r06ab11_$1.err || { tail -20 gpurun_out/r06ab11_$1.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r06ab11_$1.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$1', round(d['ms_per_step'],2), 'user kernel', round(r.get('kernel_ms') or 0,2), 'parity', (d.get('parity') or {}).get('ok'))"
}
run new_1 libblp.so "" && run prev_1 libblp_prev.so --no-parity && run new_2 libblp.so --no-parity && run prev_2 libblp_prev.so --no-parity && run new_3 libblp.so --no-parity && run prev_3 libblp_prev.so --no-parity
