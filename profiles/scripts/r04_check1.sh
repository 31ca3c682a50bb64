#!/bin/bash
# Round 4, first check: the whole GPU suite (new: at-size configs 1/3/4/5, the W=3 exchange
# compaction, concurrent short-row batch creation; knob refactor) and the default bench line
# with its exchange block.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rs --durations=15 > gpurun_out/r04c1_t1.log 2>&1 || { tail -60 gpurun_out/r04c1_t1.log; exit 1; }
tail -22 gpurun_out/r04c1_t1.log
timeout -k 10 300 python bench.py > gpurun_out/r04c1_bench.json 2> gpurun_out/r04c1_bench.err || { tail -20 gpurun_out/r04c1_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r04c1_bench.json'));print('bench', round(d['ms_per_step'],3), d['value'], d['kernels_ms'], d['parity']['ok'], d['exchange'])"
