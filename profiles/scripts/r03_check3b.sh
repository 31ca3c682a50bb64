#!/bin/bash
# Round 3, third check, part 2: e2e config 2 and config 1, config 4 (dense headline + pruned
# line, ARPACK baseline), config 5 with its at-scale parity block.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --mode e2e --config c2 > gpurun_out/c3_e2e_c2.json 2> gpurun_out/c3_e2e_c2.err || { tail -20 gpurun_out/c3_e2e_c2.err; exit 1; }
tail -1 gpurun_out/c3_e2e_c2.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print('e2e c2', round(d['e2e_s'],3), d['ok'])"
timeout -k 10 600 python bench.py --mode e2e --config yelp > gpurun_out/c3_e2e_yelp.json 2> gpurun_out/c3_e2e_yelp.err || { tail -20 gpurun_out/c3_e2e_yelp.err; exit 1; }
tail -1 gpurun_out/c3_e2e_yelp.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print('e2e yelp', round(d['e2e_s'],3), d['ok'])"
timeout -k 10 600 python bench.py --mode svd --steps 5 --warmup 1 > gpurun_out/c3_svd.json 2> gpurun_out/c3_svd.err || { tail -20 gpurun_out/c3_svd.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/c3_svd.json'));print('svd', round(d['ms_per_step'],3), d['parity'], d['pruned_topk']['ms_per_step'], d['pruned_topk']['lists_equal_dense'])"
timeout -k 10 900 python -u bench.py --mode sharded --config c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c3_c5.json 2> gpurun_out/c3_c5.err || { tail -20 gpurun_out/c3_c5.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/c3_c5.json'));print('c5', round(d['ms_per_step'],3), d['roofline'].get('kernel_ms'), d.get('parity', {}).get('ok'))"
