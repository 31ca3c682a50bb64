#!/bin/bash
# Round 6, final check 4 at HEAD: config 4 (rank-64 SVD scorer, MFMA reconstruct) and config 5
# (1B edges, row-block sharded ingest, RCCL all-gather at world 1, rank-local scoring) lines.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --mode svd > gpurun_out/r06fin4_svd.json 2> gpurun_out/r06fin4_svd.err || { tail -20 gpurun_out/r06fin4_svd.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r06fin4_svd.json').read().strip().splitlines()[-1]);print('c4', round(d['ms_per_step'],4), d['value'], d.get('parity'))"
timeout -k 10 900 python -u bench.py --mode sharded --config c5 --steps 3 --warmup 1 > gpurun_out/r06fin4_c5.json 2> gpurun_out/r06fin4_c5.err || { tail -20 gpurun_out/r06fin4_c5.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r06fin4_c5.json').read().strip().splitlines()[-1]);print('c5', round(d['ms_per_step'],2), d['value'], d.get('parity', {}).get('ok'), d.get('kernels_ms'))"
timeout -k 10 600 python bench.py --mode topk > gpurun_out/r06fin4_topk.json 2> gpurun_out/r06fin4_topk.err || { tail -20 gpurun_out/r06fin4_topk.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r06fin4_topk.json').read().strip().splitlines()[-1]);print('c3', round(d['ms_per_step'],3), d.get('parity'))"
