#!/bin/bash
# Round 5 call V: run-head grouping with an atomic active list (k_run_heads) and the item count's
# atomic active append, against the ordered scan paths (BLP_RUNS_SCAN=1 BLP_ITEM_NZ_SCAN=1);
# the grouping write's pairs per round (libblp_exp1.so -DBLP_ITEMW_U=8, libblp_exp2.so 16). The
# similarity and headline tests first; config-2 bench lines alternating; kernel stats of each.
set -o pipefail
R=$GRAFT_REPO_ROOT
L=$R/bipartite-link-prediction_amd/blp
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_similarity.py tests/test_gpu_headline.py > gpurun_out/r05v_tests.log 2>&1 || { tail -40 gpurun_out/r05v_tests.log; exit 1; }
tail -2 gpurun_out/r05v_tests.log
b() {  # name, env...
  local n=$1
  shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r05v_$n.json 2> gpurun_out/r05v_$n.err || { tail -20 gpurun_out/r05v_$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r05v_$n.json'));print('$n', round(d['ms_per_step'],3), {k:{kk:round(vv,3) for kk,vv in v.items()} for k,v in d['kernels_ms'].items()}, d['parity']['ok'])"
}
for i in 1 2 3; do
  b def_$i
  b scan_$i BLP_RUNS_SCAN=1 BLP_ITEM_NZ_SCAN=1
  b w8_$i BLP_LIB=$L/libblp_exp1.so
  b w16_$i BLP_LIB=$L/libblp_exp2.so
done
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/r05v_trace
for v in def scan; do
  rm -rf /tmp/prof_v
  if [ $v = scan ]; then export BLP_RUNS_SCAN=1 BLP_ITEM_NZ_SCAN=1; fi
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_v -o v -- python3 $R/bench.py --no-cpu-baseline --no-parity > $R/gpurun_out/r05v_trace_$v.log 2>&1 || exit 1
  for f in $(find /tmp/prof_v -name "*kernel_stats.csv"); do cp $f $R/gpurun_out/r05v_trace/${v}_kernel_stats.csv; done
done
ls $R/gpurun_out/r05v_trace
