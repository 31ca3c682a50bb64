#!/bin/bash
# config 2: short-row (business) scorer sources per dequeue (BLP_DQ_SHORT), each value twice, interleaved
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
for rep in 1 2; do
  for q in 2 3 4 6; do
    BLP_DQ_SHORT=$q timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity > gpurun_out/dq_${q}_$rep.json 2> gpurun_out/dq_${q}_$rep.err || exit 1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernels_ms']; print(sys.argv[2], round(d['ms_per_step'],3), {n:(round(v['score_ms'],3),round(v['group_ms'],3)) for n,v in k.items()}, flush=True)" gpurun_out/dq_${q}_$rep.json $q
  done
done
