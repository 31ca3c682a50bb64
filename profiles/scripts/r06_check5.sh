#!/bin/bash
# Round 6, check 5: the wedge-set tests, the new non-bipartite fallback test, the debug build's tests.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_similarity.py -k "wedge_set or general_graph" -x -v --timeout 300 --timeout-method thread > gpurun_out/r06c5_sim.log 2>&1 || { tail -40 gpurun_out/r06c5_sim.log; exit 1; }
tail -3 gpurun_out/r06c5_sim.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_debug.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06c5_debug.log 2>&1 || { tail -40 gpurun_out/r06c5_debug.log; exit 1; }
tail -2 gpurun_out/r06c5_debug.log
