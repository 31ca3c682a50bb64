#!/bin/bash
# Round 5 call AD: pairs per thread per round of the business hist and item count: experiment
# builds libblp_exp1.so (-DBLP_HIST_U=8 -DBLP_ITEMC_U=8) and libblp_exp2.so (the same with -DBLP_SCATTER_U=12); the
# similarity knob matrix under each, then config-2 bench lines alternating.
set -o pipefail
R=$GRAFT_REPO_ROOT
L=$R/bipartite-link-prediction_amd/blp
cd $R || exit 1
mkdir -p gpurun_out
for v in exp1 exp2; do
  BLP_LIB=$L/libblp_$v.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_similarity.py -k "kernel_paths or user_and_business" > gpurun_out/r05ad_tests_$v.log 2>&1 || { tail -30 gpurun_out/r05ad_tests_$v.log; exit 1; }
  tail -1 gpurun_out/r05ad_tests_$v.log
done
b() {  # name, env...
  local n=$1
  shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r05ad_$n.json 2> gpurun_out/r05ad_$n.err || { tail -20 gpurun_out/r05ad_$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r05ad_$n.json'));print('$n', round(d['ms_per_step'],3), {k:{kk:round(vv,3) for kk,vv in v.items()} for k,v in d['kernels_ms'].items()}, d['parity']['ok'])"
}
for i in 1 2 3; do
  b def_$i
  b hc8_$i BLP_LIB=$L/libblp_exp1.so
  b hc8s12_$i BLP_LIB=$L/libblp_exp2.so
done
