#!/bin/bash
# Quick config-2 bench (no CPU baseline) + optional extra args; prints the JSON line.
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/q_bench.json 2> gpurun_out/q_bench.err || { tail -30 gpurun_out/q_bench.err; exit 1; }
cat gpurun_out/q_bench.json
