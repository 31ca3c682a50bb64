#!/bin/bash
# Round 5: where similarity.main's 20-30 ms host stalls sit. Config-2 end to end twice with every
# HIP call over 3 ms reported (BLP_SLOW_HIP_MS) beside the graph stage timers; then the host-memory
# microbenchmark (pinned vs pageable fetch, allocation and free costs).
set -o pipefail
cd $GRAFT_REPO_ROOT || exit 1
mkdir -p gpurun_out
for i in 1 2; do
  BLP_SLOW_HIP_MS=3 BLP_GRAPH_PROF=1 BLP_CREATE_PROF=1 timeout -k 10 300 python bench.py --mode e2e --config c2 > gpurun_out/r05_slow_e2e_$i.json 2> gpurun_out/r05_slow_e2e_$i.err || exit 1
done
timeout -k 10 120 python profiles/scripts/r05_hostmem.py 600 > gpurun_out/r05_hostmem.json || exit 1
cat gpurun_out/r05_hostmem.json
