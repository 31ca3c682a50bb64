#!/bin/bash
# Round 5 call R: BLP_ITEM_NB=512 as the default -- the similarity and headline tests; config-2
# bench lines alternating: default (512 buckets), 2048 (the old default), 1024, and the
# co-scheduled CU share at 200 / 208 user CUs with 512 buckets.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_similarity.py tests/test_gpu_headline.py > gpurun_out/r05r_tests.log 2>&1 || { tail -40 gpurun_out/r05r_tests.log; exit 1; }
tail -2 gpurun_out/r05r_tests.log
b() {  # name, env...
  local n=$1
  shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r05r_$n.json 2> gpurun_out/r05r_$n.err || { tail -20 gpurun_out/r05r_$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r05r_$n.json'));print('$n', round(d['ms_per_step'],3), {k:{kk:round(vv,3) for kk,vv in v.items()} for k,v in d['kernels_ms'].items()}, d['parity']['ok'])"
}
for i in 1 2 3; do
  b def_$i
  b nb2048_$i BLP_ITEM_NB=2048
  b nb1024_$i BLP_ITEM_NB=1024
  b cus200_$i BLP_COSCHED_CUS=200
  b cus208_$i BLP_COSCHED_CUS=208
done
