#!/bin/bash
# Round 6, A/B 10, alternating on one box: config 5's user pass alone, k_score_split's short
# slices one pair group per wave at a time (default) against two groups in flight per wave
# (BLP_SPLIT_ILV=1: both groups' metadata, then both rows, then both groups' tests). The first
# ILV arm also checks parity. Result (r06_ab10.txt): 369 against 327 ms, slower; the knob and
# its code were removed after the run.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
run() {  # name env-assignment extra
  timeout -k 10 300 env $2 python -u bench.py --mode sharded --config c5 --sides user --steps 3 --warmup 1 --no-cpu-baseline $3 > gpurun_out/r06ab10_$1.json 2> gpurun_out/r06ab10_$1.err || { tail -20 gpurun_out/r06ab10_$1.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r06ab10_$1.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$1', round(d['ms_per_step'],2), 'kernel', round(r.get('kernel_ms') or 0,2), 'parity', (d.get('parity') or {}).get('ok'))"
}
run ilv_1 BLP_SPLIT_ILV=1 "" && run def_1 BLP_X=0 --no-parity && run ilv_2 BLP_SPLIT_ILV=1 --no-parity && run def_2 BLP_X=0 --no-parity && run ilv_3 BLP_SPLIT_ILV=1 --no-parity && run def_3 BLP_X=0 --no-parity
