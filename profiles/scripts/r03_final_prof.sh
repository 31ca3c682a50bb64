#!/bin/bash
# Round 3 final evidence: rocprofv3 kernel trace + FETCH/WRITE + SQ/TCC counter passes of the
# config-2 bench (r03_v5_bench: the name bench.py's pmc_fields picks), config 3 (r03_topk_v4)
# and config 4 (r03_svd_c4), plus the config-3 phase clocks. Summaries only come back.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
bash profiles/scripts/r03_prof.sh r03_v5_bench > gpurun_out/fp_c2.log 2>&1 || { tail -20 gpurun_out/fp_c2.log; exit 1; }
head -8 gpurun_out/r03_v5_bench.md | cut -c1-200
bash profiles/scripts/r03_prof.sh r03_topk_v4 --mode topk > gpurun_out/fp_c3.log 2>&1 || { tail -20 gpurun_out/fp_c3.log; exit 1; }
head -6 gpurun_out/r03_topk_v4.md | cut -c1-200
BLP_LIB=$R/bipartite-link-prediction_amd/blp/libblp_tkprof.so timeout -k 10 300 python profiles/scripts/topk_probe.py > gpurun_out/r03_topk_v4_phases.txt 2>&1 || { tail -5 gpurun_out/r03_topk_v4_phases.txt; exit 1; }
cat gpurun_out/r03_topk_v4_phases.txt
bash profiles/scripts/r03_prof.sh r03_svd_c4 --mode svd > gpurun_out/fp_c4.log 2>&1 || { tail -20 gpurun_out/fp_c4.log; exit 1; }
head -6 gpurun_out/r03_svd_c4.md | cut -c1-200
