#!/bin/bash
# Round 5 call Q: the business pass's grouping geometry and the grouping gate -- config-2 bench lines
# alternating: default; BLP_ITEM_NB=256 / 512 (fewer interleaved buckets: longer runs per scatter
# workgroup); BLP_GROUP_NBLK=128 (fewer scatter workgroups); BLP_PAIR_GATE=1 (the business grouping
# waits for the user grouping); then kernel traces of two of them.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
b() {  # name, env...
  local n=$1
  shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r05q_$n.json 2> gpurun_out/r05q_$n.err || { tail -20 gpurun_out/r05q_$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r05q_$n.json'));print('$n', round(d['ms_per_step'],3), {k:{kk:round(vv,3) for kk,vv in v.items()} for k,v in d['kernels_ms'].items()}, d['parity']['ok'])"
}
for i in 1 2; do
  b def_$i
  b nb256_$i BLP_ITEM_NB=256
  b nb512_$i BLP_ITEM_NB=512
  b nblk128_$i BLP_GROUP_NBLK=128
  b gate_$i BLP_PAIR_GATE=1
  b gate_nb256_$i BLP_PAIR_GATE=1 BLP_ITEM_NB=256
done
cd /tmp && export TMPDIR=/tmp
for v in nb256 gate; do
  rm -rf /tmp/prof_q
  if [ $v = nb256 ]; then export BLP_ITEM_NB=256; unset BLP_PAIR_GATE; else export BLP_PAIR_GATE=1; unset BLP_ITEM_NB; fi
  timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_q -o q -- python3 $R/bench.py --no-cpu-baseline --no-parity --steps 3 --warmup 1 > $R/gpurun_out/r05q_trace_$v.log 2>&1 || exit 1
  mkdir -p $R/gpurun_out/r05q_trace
  for f in $(find /tmp/prof_q -name "*kernel_trace.csv"); do gzip -c $f > $R/gpurun_out/r05q_trace/${v}_$(basename $f).gz; done
done
ls $R/gpurun_out/r05q_trace
