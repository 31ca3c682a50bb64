#!/bin/bash
# Round 5 A/B 2: the business grouping write -- 8-byte stage with row bounds (default),
# the 16-byte stage (BLP_GROUP_ROWS16=1), y only with the scorer gathering rows (BLP_GROUP_YN=1) --
# alternating on one box; then the similarity GPU tests (device planning) and config 2 end to end.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_similarity.py tests/test_gpu_headline.py tests/test_gpu_debug.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05ab2_tests.log 2>&1 || { tail -60 gpurun_out/r05ab2_tests.log; exit 1; }
tail -2 gpurun_out/r05ab2_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r05ab2_parity.json 2> gpurun_out/r05ab2_parity.err || { tail -20 gpurun_out/r05ab2_parity.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r05ab2_parity.json'));print('parity bench', round(d['ms_per_step'],3), d['kernels_ms'], d['parity']['ok'], d['including_batch_create'])"
for i in 1 2 3; do
  for v in s8 s16 yn; do
    unset BLP_GROUP_ROWS16 BLP_GROUP_YN
    if [ $v = s16 ]; then export BLP_GROUP_ROWS16=1; fi
    if [ $v = yn ]; then export BLP_GROUP_YN=1; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity --steps 30 > gpurun_out/r05ab2_${v}_$i.json 2> gpurun_out/r05ab2_${v}_$i.err || { tail -20 gpurun_out/r05ab2_${v}_$i.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r05ab2_${v}_$i.json'));print('$v', $i, round(d['ms_per_step'],3), {k:{a:round(b,3) for a,b in v.items()} for k,v in d['kernels_ms'].items()}, round(d['including_batch_create']['batch_create_s'],4))"
  done
done
unset BLP_GROUP_ROWS16 BLP_GROUP_YN
for i in 1 2; do
  BLP_CREATE_PROF=1 timeout -k 10 300 python bench.py --mode e2e --config c2 > gpurun_out/r05ab2_e2e_$i.json 2> gpurun_out/r05ab2_e2e_$i.err || { tail -20 gpurun_out/r05ab2_e2e_$i.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r05ab2_e2e_$i.json').read().strip().splitlines()[-1]);print('e2e', round(d['e2e_s'],4), {k: round(v,4) for k,v in d['phases_s'].items()}, d['ok'])"
done
grep "blp_batch_create" gpurun_out/r05ab2_e2e_2.err | head -20
