#!/bin/bash
# Round 6, A/B 2, alternating on one box: (1) what a pinned staging ring costs (r06_pinned_probe);
# (2) the config-2 step with k_score_short's header prefetch (pf build) at other CU shares for the
# user pass (BLP_COSCHED_CUS; the default picks 192), against the default build.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 120 ./profiles/scripts/r06_pinned_probe > gpurun_out/r06ab2_pinned.txt 2>&1 || { cat gpurun_out/r06ab2_pinned.txt; exit 1; }
cat gpurun_out/r06ab2_pinned.txt
L=$R/bipartite-link-prediction_amd/blp
for round in 1 2; do
  for v in def:0 pf:0 pf:200 pf:208 pf:216 def:200; do
    name=${v%%:*}; cus=${v##*:}
    lib=$L/libblp.so
    [ $name != def ] && lib=$L/libblp_$name.so
    env=""
    [ $cus != 0 ] && env="BLP_COSCHED_CUS=$cus"
    env $env BLP_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-exchange --no-parity > gpurun_out/r06ab2_${name}_${cus}_$round.json 2> gpurun_out/r06ab2_${name}_${cus}_$round.err || { tail -20 gpurun_out/r06ab2_${name}_${cus}_$round.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r06ab2_${name}_${cus}_$round.json'));print('$name', $cus, $round, round(d['ms_per_step'],4), {k: {kk: round(vv, 4) for kk, vv in x.items()} for k, x in d['kernels_ms'].items()})"
  done
done
