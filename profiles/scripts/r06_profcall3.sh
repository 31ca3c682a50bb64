#!/bin/bash
# Round 6, profile call 3: config 2 at HEAD (after the direct row lookup and the fused run
# grouping): trace, FETCH_SIZE, WRITE_SIZE, SQ and TCC passes (r06_prof.sh -> r06_v2_bench).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
bash profiles/scripts/r06_prof.sh r06_v2_bench 300 --no-exchange || exit 1
