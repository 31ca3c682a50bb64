#!/bin/bash
# prefault of the score fetch buffers: the similarity suite, then config 2 end to end x3
set -o pipefail
mkdir -p gpurun_out/c19
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_similarity.py tests/test_gpu_ingest.py > gpurun_out/c19/t.txt 2>&1 || { tail -40 gpurun_out/c19/t.txt; exit 1; }
tail -2 gpurun_out/c19/t.txt
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --mode e2e --config c2 > gpurun_out/c19/e2e_$i.json 2> gpurun_out/c19/e2e_$i.err || { tail -20 gpurun_out/c19/e2e_$i.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/c19/e2e_$i.json').read().strip().splitlines()[-1]);print('e2e', round(d['e2e_s'],4), {k: round(v,4) for k,v in d['phases_s'].items()}, d['ok'])"
done
