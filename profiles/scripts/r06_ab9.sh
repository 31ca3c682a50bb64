#!/bin/bash
# Round 6, A/B 9, alternating on one box: config 5's business pass alone (--sides business), the
# hash-set routing bound (BLP_HASH_WORK build ids; default 8192 = half the 16K-slot table) and the
# 128 KiB-table variant (BLP_HASH_BIG), re-measured after the source partition and 4-source claims.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
run() {  # name env-assignment
  timeout -k 10 300 env $2 python -u bench.py --mode sharded --config c5 --sides business --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-exchange > gpurun_out/r06ab9_$1.json 2> gpurun_out/r06ab9_$1.err || { tail -20 gpurun_out/r06ab9_$1.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r06ab9_$1.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$1', round(d['ms_per_step'],2), 'plan', r.get('plan',{}).get('hash_sources'))"
}
for round in 1 2; do
  run def_$round BLP_X=0 && run w4k_$round BLP_HASH_WORK=4096 && run w6k_$round BLP_HASH_WORK=6144 && run w11k_$round BLP_HASH_WORK=11000 && run big_$round BLP_HASH_BIG=1 || exit 1
done
