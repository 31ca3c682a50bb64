#!/bin/bash
# device graph.txt parse: parity tests, the suites that load graph.txt, then end to end x2
set -o pipefail
mkdir -p gpurun_out/c15
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ingest.py \
  -k "device_parse or load_edge_list" > gpurun_out/c15/t1.txt 2>&1 || { tail -40 gpurun_out/c15/t1.txt; exit 1; }
tail -3 gpurun_out/c15/t1.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ingest.py \
  tests/test_gpu_similarity.py > gpurun_out/c15/t2.txt 2>&1 || { tail -40 gpurun_out/c15/t2.txt; exit 1; }
tail -3 gpurun_out/c15/t2.txt
for i in 1 2; do
  BLP_GRAPH_PROF=1 BLP_INGEST_PROF=1 timeout -k 10 300 python bench.py --mode e2e --config c2 > gpurun_out/c15/e2e_$i.json 2> gpurun_out/c15/e2e_$i.err || { tail -20 gpurun_out/c15/e2e_$i.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/c15/e2e_$i.json').read().strip().splitlines()[-1]);print('e2e', round(d['e2e_s'],4), {k: round(v,4) for k,v in d['phases_s'].items()}, d['graph_phase_detail_s'], d['ok'])"
done
