#!/bin/bash
# GPU suite, then config 5 (row-block sharded ingest + device CSR + chunk-parallel scoring) at 1 GPU.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_gputest.log 2>&1 || { tail -40 gpurun_out/r02_gputest.log; exit 1; }
tail -2 gpurun_out/r02_gputest.log
timeout -k 10 900 python -u bench.py --mode sharded --config c5 --steps 5 --warmup 1 > gpurun_out/r02_c5.json 2> gpurun_out/r02_c5.err || { tail -30 gpurun_out/r02_c5.err; exit 1; }
cat gpurun_out/r02_c5.json
