#!/bin/bash
# Round 5 A/B 3: config 2's business pass -- the three-barrier short-row scorer with the 8-byte-stage
# grouping (default) against the segment scorer (BLP_SHORT_SEG=1) and the 16-byte-stage grouping
# (BLP_GROUP_ROWS16=1), alternating on one box; the similarity tests first; config 2 end to end
# with the device planning pass; then the LDS bank-conflict attribution of the user scorer.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_similarity.py tests/test_gpu_headline.py tests/test_gpu_debug.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05ab3_tests.log 2>&1 || { tail -60 gpurun_out/r05ab3_tests.log; exit 1; }
tail -2 gpurun_out/r05ab3_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r05ab3_parity.json 2> gpurun_out/r05ab3_parity.err || { tail -20 gpurun_out/r05ab3_parity.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r05ab3_parity.json'));print('parity bench', round(d['ms_per_step'],3), d['kernels_ms'], d['parity']['ok'], d['including_batch_create'])"
for i in 1 2; do
  for v in three seg s16; do
    unset BLP_SHORT_SEG BLP_GROUP_ROWS16
    if [ $v = seg ]; then export BLP_SHORT_SEG=1; fi
    if [ $v = s16 ]; then export BLP_GROUP_ROWS16=1; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity --no-exchange --steps 30 > gpurun_out/r05ab3_${v}_$i.json 2> gpurun_out/r05ab3_${v}_$i.err || { tail -20 gpurun_out/r05ab3_${v}_$i.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r05ab3_${v}_$i.json'));print('$v', $i, round(d['ms_per_step'],3), {k:{a:round(b,3) for a,b in v.items()} for k,v in d['kernels_ms'].items()}, round(d['including_batch_create']['batch_create_s'],4))"
  done
done
unset BLP_SHORT_SEG BLP_GROUP_ROWS16
for v in three seg; do
  unset BLP_SHORT_SEG
  if [ $v = seg ]; then export BLP_SHORT_SEG=1; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity --no-exchange --steps 30 --sides business > gpurun_out/r05ab3_alone_${v}.json 2> gpurun_out/r05ab3_alone_${v}.err || { tail -20 gpurun_out/r05ab3_alone_${v}.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r05ab3_alone_${v}.json'));print('business alone $v', round(d['ms_per_step'],3), d['kernels_ms'])"
done
unset BLP_SHORT_SEG
for i in 1 2; do
  BLP_CREATE_PROF=1 BLP_GRAPH_PROF=1 timeout -k 10 300 python bench.py --mode e2e --config c2 > gpurun_out/r05ab3_e2e_$i.json 2> gpurun_out/r05ab3_e2e_$i.err || { tail -20 gpurun_out/r05ab3_e2e_$i.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r05ab3_e2e_$i.json').read().strip().splitlines()[-1]);print('e2e', round(d['e2e_s'],4), {k: round(v,4) for k,v in d['phases_s'].items()}, d['graph_phase_detail_s'], d['ok'])"
done
grep -E "blp_batch_create|graph_finish|codes" gpurun_out/r05ab3_e2e_2.err | head -40
bash profiles/scripts/r05_lds_attr.sh
