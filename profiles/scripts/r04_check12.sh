#!/bin/bash
# Round 4, check 12: the co-scheduled CU share of the user scorer re-measured after this round's
# scorer changes (BLP_COSCHED_CUS = 184 / 192 / 200 / 208, two rounds, config-2 step).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
ab() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --no-exchange --steps 20 --warmup 3 --no-parity > gpurun_out/ab12_$name.json 2> gpurun_out/ab12_$name.err || { tail -5 gpurun_out/ab12_$name.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab12_$name.json'));print('$name', round(d['ms_per_step'],4), {k: (round(v['score_ms'],3), round(v['group_ms'],3)) for k,v in d['kernels_ms'].items()})"
}
for r in a b; do
  for c in 184 192 200 208; do ab cus${c}$r BLP_COSCHED_CUS=$c || exit 1; done
done
