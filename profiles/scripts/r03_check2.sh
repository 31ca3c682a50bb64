#!/bin/bash
# Round 3, second check after the grouping / hop-3 / top-k / loader changes: the whole GPU suite
# on the release build, smoke(), then the default bench line, config 3 (parity), e2e config 2
# and config 1, and config 5 with its at-scale parity block.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/c2_gputest.log 2>&1 || { tail -40 gpurun_out/c2_gputest.log; exit 1; }
tail -2 gpurun_out/c2_gputest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/c2_smoke.log 2>&1 || { tail -20 gpurun_out/c2_smoke.log; exit 1; }
tail -1 gpurun_out/c2_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/c2_bench.json 2> gpurun_out/c2_bench.err || { tail -20 gpurun_out/c2_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/c2_bench.json'));print('bench', round(d['ms_per_step'],3), d['value'], d['kernels_ms'], d['setup_s'], d['parity']['u_cn_exact'], d['cpu_baseline'])"
timeout -k 10 300 python bench.py --mode topk --steps 5 --warmup 1 > gpurun_out/c2_topk.json 2> gpurun_out/c2_topk.err || { tail -20 gpurun_out/c2_topk.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/c2_topk.json'));print('topk', round(d['ms_per_step'],3), d['work'], d['parity'])"
BLP_INGEST_PROF=1 timeout -k 10 600 python bench.py --mode e2e --config c2 > gpurun_out/c2_e2e_c2.json 2> gpurun_out/c2_e2e_c2.err || { tail -20 gpurun_out/c2_e2e_c2.err; exit 1; }
tail -1 gpurun_out/c2_e2e_c2.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print('e2e c2', round(d['e2e_s'],3), d['phases_s'], d['ok'])"
grep blp_edges_load gpurun_out/c2_e2e_c2.err || true
timeout -k 10 600 python bench.py --mode e2e --config yelp > gpurun_out/c2_e2e_yelp.json 2> gpurun_out/c2_e2e_yelp.err || { tail -20 gpurun_out/c2_e2e_yelp.err; exit 1; }
tail -1 gpurun_out/c2_e2e_yelp.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print('e2e yelp', round(d['e2e_s'],3), d['phases_s'], d['ok'])"
timeout -k 10 900 python -u bench.py --mode sharded --config c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c2_c5.json 2> gpurun_out/c2_c5.err || { tail -20 gpurun_out/c2_c5.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/c2_c5.json'));print('c5', round(d['ms_per_step'],3), d['roofline'].get('kernel_ms'), d['roofline'].get('limiter'), d.get('parity', {}).get('ok'))"
