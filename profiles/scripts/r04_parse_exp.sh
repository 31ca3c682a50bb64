#!/bin/bash
# host graph.txt parse micro-benchmark on the GPU box's host cores (no GPU use)
set -e
mkdir -p gpurun_out/pt
cd bipartite-link-prediction_amd
timeout -k 10 120 python - <<'PY'
import sys, os
sys.path.insert(0, '.')
from blp import synth
U, B, D = synth.CONFIGS['c2']
u, b = synth.review_edges(U, B, D, seed=0)
with open('/tmp/graph_c2.txt', 'w') as f:
    f.write('\n'.join('%d %d' % (x, y) for x, y in zip(u.tolist(), b.tolist())))
    f.write('\n')
print(os.path.getsize('/tmp/graph_c2.txt'))
PY
cd ..
g++ -O3 -pthread profiles/scripts/r04_parse_microbench.cpp -o /tmp/pmb
for m in 0 1 2 3; do for nt in 1 8 16; do timeout -k 5 60 /tmp/pmb /tmp/graph_c2.txt $nt $m; done; done > gpurun_out/pt/micro.txt 2>&1
cd bipartite-link-prediction_amd
for i in 1 2 3 4; do BLP_INGEST_PROF=1 timeout -k 5 60 python -c "
import sys,ctypes,time; sys.path.insert(0,'.')
from blp._lib import lib, check
h=ctypes.c_void_p(); t=time.perf_counter(); check(lib().blp_edges_load(b'/tmp/graph_c2.txt',0,1,ctypes.byref(h))); print('load %.4f'%(time.perf_counter()-t))
"; done > ../gpurun_out/pt/load.txt 2>&1
echo done
cd ..
for i in 1 2; do
  BLP_GRAPH_PROF=1 BLP_INGEST_PROF=1 timeout -k 10 300 python bench.py --mode e2e --config c2 > gpurun_out/pt/e2e_$i.json 2> gpurun_out/pt/e2e_$i.err || { tail -20 gpurun_out/pt/e2e_$i.err; exit 1; }
done
echo e2e done
