#!/bin/bash
# Round 5 call D: the THP A/B of config-2 similarity.main (r05_thp_ab.sh), the config-3 top-k
# phase clocks with per-method selection rounds (libblp_tkprof.so, -DBLP_PROF), then profile B
# (config-5 business pass, config-3 top-k).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 180 python profiles/scripts/r05_evict.py > gpurun_out/r05_evict.json || exit 1
cat gpurun_out/r05_evict.json
bash profiles/scripts/r05_thp_ab.sh || exit 1
BLP_LIB=$R/bipartite-link-prediction_amd/blp/libblp_tkprof.so timeout -k 10 300 python profiles/scripts/topk_probe.py > gpurun_out/r05_topk_phases.txt 2>&1 || { tail gpurun_out/r05_topk_phases.txt; exit 1; }
cat gpurun_out/r05_topk_phases.txt
bash profiles/scripts/r05_profB.sh
