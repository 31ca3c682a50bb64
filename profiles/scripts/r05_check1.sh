#!/bin/bash
# Round 5, check 1: the whole GPU suite (new: the 1B-draw config-5 exchange test, the pre-launch
# pointer check, the pinned headline kernels), then the default bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 400 --timeout-method thread -rs > gpurun_out/r05c1_gputest.log 2>&1 || { tail -80 gpurun_out/r05c1_gputest.log; exit 1; }
tail -3 gpurun_out/r05c1_gputest.log
grep "config5 1B" gpurun_out/r05c1_gputest.log
timeout -k 10 300 python bench.py > gpurun_out/r05c1_bench.json 2> gpurun_out/r05c1_bench.err || { tail -20 gpurun_out/r05c1_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r05c1_bench.json'));print('bench', round(d['ms_per_step'],3), d['value'], d['kernels_ms'], d['parity']['ok'])"
