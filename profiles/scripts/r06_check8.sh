#!/bin/bash
# Round 6, check 8: the graph-stream event queued after the pair upload in blp_batch_create (the
# upload's host syncs no longer wait for the graph build's last kernels). Similarity tests, the
# config-1 similarity.main test, then similarity.main at configs 1 and 2 with the creation stages.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_similarity.py tests/test_gpu_headline.py tests/test_gpu_atsize.py -k "not config5 and not config3 and not config4" -x -q --timeout 300 --timeout-method thread > gpurun_out/r06c8_tests.log 2>&1 || { tail -30 gpurun_out/r06c8_tests.log; exit 1; }
tail -1 gpurun_out/r06c8_tests.log
for c in yelp yelp c2 c2; do
  BLP_CREATE_PROF=1 timeout -k 10 300 python bench.py --mode e2e --config $c > gpurun_out/r06c8_e2e_$c.json 2> gpurun_out/r06c8_e2e_$c.err || { tail -20 gpurun_out/r06c8_e2e_$c.err; exit 1; }
  python -c "import json;t=open('gpurun_out/r06c8_e2e_$c.json').read();d=json.loads(t[t.index('{\"metric\"'):].strip().splitlines()[0]);print('e2e $c', round(d['e2e_s'],4), d['ok'], {k: round(v,4) for k,v in d['phases_s'].items() if k in ('graph','score','score_create','files','teardown')})"
  grep "upload" gpurun_out/r06c8_e2e_$c.err | head -4 || true
done
