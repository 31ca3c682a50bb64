#!/bin/bash
# Round 4, check 2 (after the long-slice queue fix): the whole GPU suite, the default bench line
# with its exchange block, and config 2 end to end with blp_batch_create's stage times.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rs --durations=15 > gpurun_out/r04c2_gputest.log 2>&1 || { tail -60 gpurun_out/r04c2_gputest.log; exit 1; }
tail -22 gpurun_out/r04c2_gputest.log
timeout -k 10 300 python bench.py > gpurun_out/r04c2_bench.json 2> gpurun_out/r04c2_bench.err || { tail -20 gpurun_out/r04c2_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r04c2_bench.json'));print('bench', round(d['ms_per_step'],3), d['value'], d['kernels_ms'], d['parity']['ok'], d['exchange'])"
BLP_CREATE_PROF=1 timeout -k 10 300 python bench.py --mode e2e --config c2 > gpurun_out/r04c2_e2e.json 2> gpurun_out/r04c2_e2e.err || { tail -20 gpurun_out/r04c2_e2e.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r04c2_e2e.json'));print('e2e', d['e2e_s'], d['phases_s'], d['ok'])"
grep "blp_batch_create" gpurun_out/r04c2_e2e.err | tail -24
