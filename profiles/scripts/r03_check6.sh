#!/bin/bash
# Round 3, final check after the hash-set scorer claims 4 sources at a time: the whole GPU
# suite on the release build, smoke(), the default bench line, config 3, config 5 with parity.
# (No profiling: r03_c5_v3 and r03_c5_business_v4 are the profiles of this code.)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rs > gpurun_out/c6_gputest.log 2>&1 || { tail -40 gpurun_out/c6_gputest.log; exit 1; }
tail -3 gpurun_out/c6_gputest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/c6_smoke.log 2>&1 || { tail -20 gpurun_out/c6_smoke.log; exit 1; }
tail -1 gpurun_out/c6_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/c6_bench.json 2> gpurun_out/c6_bench.err || { tail -20 gpurun_out/c6_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/c6_bench.json'));print('bench', round(d['ms_per_step'],3), d['value'], d['kernels_ms'], d['parity']['u_cn_exact'], d['cpu_baseline'])"
timeout -k 10 300 python bench.py --mode topk --steps 5 --warmup 1 > gpurun_out/c6_topk.json 2> gpurun_out/c6_topk.err || { tail -20 gpurun_out/c6_topk.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/c6_topk.json'));print('topk', round(d['ms_per_step'],3), d['parity'])"
timeout -k 10 900 python -u bench.py --mode sharded --config c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c6_c5.json 2> gpurun_out/c6_c5.err || { tail -20 gpurun_out/c6_c5.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/c6_c5.json'));print('c5', round(d['ms_per_step'],3), d['roofline'].get('kernel_ms'), d.get('parity', {}).get('ok'))"
