#!/bin/bash
# Round 6, profile call 4 (first the timer tests): config 2 at HEAD (end of round: the two-launch run grouping and the two-stage row
# prefetch): trace, FETCH_SIZE, WRITE_SIZE, SQ and TCC passes (r06_prof.sh -> r06_v3_bench).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_similarity.py -k "totals_follow or repeat_is_deterministic or kernel_paths" -x -q --timeout 120 --timeout-method thread > gpurun_out/r06pc4_tests.log 2>&1 || { tail -30 gpurun_out/r06pc4_tests.log; exit 1; }
tail -1 gpurun_out/r06pc4_tests.log
bash profiles/scripts/r06_prof.sh r06_v3_bench 300 --no-exchange || exit 1
