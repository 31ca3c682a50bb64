#!/bin/bash
# Round 4, experiment 1: config-2 user side alone -- the LARGE block scorer (one 125 KB bitmap,
# one workgroup per CU) against the chunk-parallel scorer on two half-universe chunks (64 KiB
# bitmaps: two workgroups per CU with BLP_SPLIT_BIG=0; one with the 128 KiB kernel).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
q() {  # name, env..., -- bench args
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --sides user --no-cpu-baseline --no-exchange --steps 10 --warmup 2 > gpurun_out/e1_$name.json 2> gpurun_out/e1_$name.err || { tail -5 gpurun_out/e1_$name.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/e1_$name.json'));print('$name', round(d['ms_per_step'],3), d['kernels_ms'], d.get('parity',{}).get('ok'), d['roofline'].get('kernel'))"
}
q base BLP_X=0 || exit 1
q split2_64k BLP_SPLIT=2 BLP_SPLIT_BIG=0 BLP_NO_HASH=1 || exit 1
q split2_128k BLP_SPLIT=2 BLP_NO_HASH=1 || exit 1
q split2_64k_short0 BLP_SPLIT=2 BLP_SPLIT_BIG=0 BLP_NO_HASH=1 BLP_SPLIT_SHORT=0 || exit 1
