#!/bin/bash
# Round 6, check 6: the whole GPU suite and smoke at HEAD after the split scorer's accumulator
# layout and branch-free short slices and the flat-load-free AA terms; then the config-2 bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06c6_gputest.log 2>&1 || { tail -40 gpurun_out/r06c6_gputest.log; exit 1; }
tail -3 gpurun_out/r06c6_gputest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06c6_smoke.log 2>&1 || { tail -20 gpurun_out/r06c6_smoke.log; exit 1; }
tail -1 gpurun_out/r06c6_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r06c6_bench.json 2> gpurun_out/r06c6_bench.err || { tail -20 gpurun_out/r06c6_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r06c6_bench.json'));print('bench', round(d['ms_per_step'],4), d['value'], d['kernels_ms'], d['parity']['ok'])"
