#!/bin/bash
# Round 3: config 5, each pass alone under a kernel trace (which kernels the 447 ms user pass and
# the 301 ms business pass are made of).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
bash profiles/scripts/r03_trace.sh r03_c5_user --mode sharded --config c5 --steps 2 --warmup 1 --sides user || exit 1
bash profiles/scripts/r03_trace.sh r03_c5_business --mode sharded --config c5 --steps 2 --warmup 1 --sides business || exit 1
