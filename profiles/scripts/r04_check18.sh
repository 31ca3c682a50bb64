#!/bin/bash
# stage timers of the graph phase (BLP_GRAPH_PROF) at config 2, and config 1 (Yelp-sized) end to end
set -o pipefail
mkdir -p gpurun_out/c18
for i in 1 2; do
  BLP_GRAPH_PROF=1 timeout -k 10 300 python bench.py --mode e2e --config c2 > gpurun_out/c18/e2e_$i.json 2> gpurun_out/c18/e2e_$i.err || { tail -20 gpurun_out/c18/e2e_$i.err; exit 1; }
  grep -E "graph_finish|codes" gpurun_out/c18/e2e_$i.err
  python -c "import json;d=json.loads(open('gpurun_out/c18/e2e_$i.json').read().strip().splitlines()[-1]);print('e2e', round(d['e2e_s'],4), {k: round(v,4) for k,v in d['phases_s'].items()}, {k: round(v,4) for k,v in d['graph_phase_detail_s'].items()}, d['ok'])"
done
timeout -k 10 300 python bench.py --mode e2e --config yelp > gpurun_out/c18/e2e_yelp.json 2> gpurun_out/c18/e2e_yelp.err || { tail -20 gpurun_out/c18/e2e_yelp.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/c18/e2e_yelp.json').read().strip().splitlines()[-1]);print('yelp', round(d['e2e_s'],4), {k: round(v,4) for k,v in d['phases_s'].items()}, d['ok'])"
