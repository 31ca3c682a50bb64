#!/bin/bash
# Round 6, check 1: the ingest upload through the pinned staging ring; the whole GPU suite, smoke(),
# the default bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ingest.py tests/test_gpu_headline.py -x -v --timeout 240 --timeout-method thread -rs > gpurun_out/r06c1_first.log 2>&1 || { tail -60 gpurun_out/r06c1_first.log; exit 1; }
tail -3 gpurun_out/r06c1_first.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rs > gpurun_out/r06c1_gputest.log 2>&1 || { tail -60 gpurun_out/r06c1_gputest.log; exit 1; }
tail -3 gpurun_out/r06c1_gputest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06c1_smoke.log 2>&1 || { tail -20 gpurun_out/r06c1_smoke.log; exit 1; }
tail -1 gpurun_out/r06c1_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r06c1_bench.json 2> gpurun_out/r06c1_bench.err || { tail -20 gpurun_out/r06c1_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r06c1_bench.json'));print('bench', round(d['ms_per_step'],3), d['value'], d['kernels_ms'], d['parity']['ok'])"
