#!/bin/bash
# Round 5 call K: the ingest / CSR tests after the double-buffer sort and the parse buffers sized
# for its reuse; then config-2 similarity.main four times (slow HIP calls logged) and config 5's
# exchange test (its CSR build).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ingest.py tests/test_gpu_similarity.py -k "csr or parse or ingest or load or cache or prewarm or main" > gpurun_out/r05k_tests.log 2>&1 || { tail -40 gpurun_out/r05k_tests.log; exit 1; }
tail -2 gpurun_out/r05k_tests.log
for i in 1 2 3 4; do
  BLP_SLOW_HIP_MS=3 BLP_GRAPH_PROF=1 timeout -k 10 300 python bench.py --mode e2e --config c2 > gpurun_out/r05k_e2e_$i.json 2> gpurun_out/r05k_e2e_$i.err || { tail -20 gpurun_out/r05k_e2e_$i.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r05k_e2e_$i.json').read().strip().splitlines()[-1]);print('e2e', round(d['e2e_s'],4), {k: round(v,4) for k,v in d['phases_s'].items()}, d['ok'])"
done
