#!/bin/bash
# Round 5 call AF: the business scatter without its 4-byte key array (BLP_NO_KEYS=1: half the open
# write streams per block; the item counts read the records' x) against the default; the knob
# matrix similarity tests, then config-2 bench lines alternating.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_similarity.py -k "kernel_paths" > gpurun_out/r05af_tests.log 2>&1 || { tail -30 gpurun_out/r05af_tests.log; exit 1; }
tail -1 gpurun_out/r05af_tests.log
b() {  # name, env...
  local n=$1
  shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r05af_$n.json 2> gpurun_out/r05af_$n.err || { tail -20 gpurun_out/r05af_$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r05af_$n.json'));print('$n', round(d['ms_per_step'],3), {k:{kk:round(vv,3) for kk,vv in v.items()} for k,v in d['kernels_ms'].items()}, d['parity']['ok'])"
}
for i in 1 2 3; do
  b def_$i
  b nokeys_$i BLP_NO_KEYS=1
done
