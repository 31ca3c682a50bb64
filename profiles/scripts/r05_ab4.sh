#!/bin/bash
# Round 5 A/B 4: (1) the co-scheduled CU share re-swept with the three-barrier business scorer
# (BLP_COSCHED_CUS 184..224); (2) k_score_short at 8 workgroups per CU (libblp_exp3.so,
# -DBLP_SHORT_MINB=8) against 7; (3) the LDS bank-conflict attribution of the user scorer.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
run() {  # name, env...
  local n=$1
  shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity --no-exchange --steps 30 > gpurun_out/r05ab4_$n.json 2> gpurun_out/r05ab4_$n.err || { tail -20 gpurun_out/r05ab4_$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r05ab4_$n.json'));print('$n', round(d['ms_per_step'],3), {k:{a:round(b,3) for a,b in v.items()} for k,v in d['kernels_ms'].items()})"
}
for i in 1 2; do
  run def_$i
  for c in 184 200 208 216 224; do run cus${c}_$i BLP_COSCHED_CUS=$c; done
  run minb8_$i BLP_LIB=$R/bipartite-link-prediction_amd/blp/libblp_exp3.so
done
bash profiles/scripts/r05_lds_attr.sh
