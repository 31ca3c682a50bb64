#!/bin/bash
# config 2: user-scorer CU share sweep (BLP_COSCHED_CUS), each share twice, interleaved
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
for rep in 1 2; do
  for c in 176 184 192 200; do
    BLP_COSCHED_CUS=$c timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity > gpurun_out/cs_${c}_$rep.json 2> gpurun_out/cs_${c}_$rep.err || exit 1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernels_ms']; print(sys.argv[2], round(d['ms_per_step'],3), {n:(round(v['score_ms'],3),round(v['group_ms'],3)) for n,v in k.items()}, flush=True)" gpurun_out/cs_${c}_$rep.json $c
  done
done
