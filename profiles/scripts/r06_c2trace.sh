#!/bin/bash
# Round 6: config-2 kernel trace of the timed steps (timeline: per-step kernel order, gaps and
# overlap of the two passes across steps). The database is analysed on the CPU side.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r06c2trace -o c2 -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-parity --no-exchange > gpurun_out/r06c2trace.json 2> gpurun_out/r06c2trace.err || { tail -20 gpurun_out/r06c2trace.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r06c2trace.json'));print('bench', round(d['ms_per_step'],4))"
