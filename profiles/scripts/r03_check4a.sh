#!/bin/bash
# Round 3, fourth check (after the wave-by-wave split scorer): the whole GPU suite on the
# release build, smoke(), the default bench line, config 3.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rs > gpurun_out/c4_gputest.log 2>&1 || { tail -40 gpurun_out/c4_gputest.log; exit 1; }
tail -3 gpurun_out/c4_gputest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/c4_smoke.log 2>&1 || { tail -20 gpurun_out/c4_smoke.log; exit 1; }
tail -1 gpurun_out/c4_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/c4_bench.json 2> gpurun_out/c4_bench.err || { tail -20 gpurun_out/c4_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/c4_bench.json'));print('bench', round(d['ms_per_step'],3), d['value'], d['kernels_ms'], d['parity']['u_cn_exact'], d['cpu_baseline'])"
timeout -k 10 300 python bench.py --mode topk --steps 5 --warmup 1 > gpurun_out/c4_topk.json 2> gpurun_out/c4_topk.err || { tail -20 gpurun_out/c4_topk.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/c4_topk.json'));print('topk', round(d['ms_per_step'],3), d['parity'])"
