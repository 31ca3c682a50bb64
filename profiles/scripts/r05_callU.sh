#!/bin/bash
# Round 5 call U: pairs per thread per round of the grouping write (k_item_write_ids): experiment
# builds libblp_exp1.so (-DBLP_ITEMW_U=8) and libblp_exp2.so (16) against the default (4; the scatter at 8 now);
# config-2 bench lines alternating, then a kernel trace of each.
set -o pipefail
R=$GRAFT_REPO_ROOT
L=$R/bipartite-link-prediction_amd/blp
cd $R || exit 1
mkdir -p gpurun_out
b() {  # name, env...
  local n=$1
  shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r05u_$n.json 2> gpurun_out/r05u_$n.err || { tail -20 gpurun_out/r05u_$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r05u_$n.json'));print('$n', round(d['ms_per_step'],3), {k:{kk:round(vv,3) for kk,vv in v.items()} for k,v in d['kernels_ms'].items()}, d['parity']['ok'])"
}
for i in 1 2 3; do
  b def_$i
  b u8_$i BLP_LIB=$L/libblp_exp1.so
  b u16_$i BLP_LIB=$L/libblp_exp2.so
done
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/r05u_trace
for v in def u8 u16; do
  rm -rf /tmp/prof_u
  LIB=$L/libblp.so
  [ $v = u8 ] && LIB=$L/libblp_exp1.so
  [ $v = u16 ] && LIB=$L/libblp_exp2.so
  BLP_LIB=$LIB timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_u -o u -- python3 $R/bench.py --no-cpu-baseline --no-parity > $R/gpurun_out/r05u_trace_$v.log 2>&1 || exit 1
  for f in $(find /tmp/prof_u -name "*kernel_stats.csv"); do cp $f $R/gpurun_out/r05u_trace/${v}_kernel_stats.csv; done
done
ls $R/gpurun_out/r05u_trace
