#!/bin/bash
# Round 6, A/B 8, alternating on one box: config 5, k_score_split's exact-AA accumulators
# interleaved per pair ([pair][2], BLP_SPLIT_AOS=1, the round-5 layout) against all low words then
# all high words (the default now). The first arm also checks parity against the oracle.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
run() {  # name env-assignment extra-args
  local n=$1; shift
  env $1 timeout -k 10 400 python -u bench.py --mode sharded --config c5 --steps 3 --warmup 1 --no-cpu-baseline $2 > gpurun_out/r06ab8_$n.json 2> gpurun_out/r06ab8_$n.err || { tail -20 gpurun_out/r06ab8_$n.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r06ab8_$n.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$n', round(d['ms_per_step'],2), 'kernel', round(r.get('kernel_ms') or 0,2), 'parity', (d.get('parity') or {}).get('ok'))"
}
run soa_1 BLP_X=0 "" && run aos_1 BLP_SPLIT_AOS=1 "--no-parity" && run soa_2 BLP_X=0 "--no-parity" && run aos_2 BLP_SPLIT_AOS=1 "--no-parity"
