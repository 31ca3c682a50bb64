#!/bin/bash
# Round 4, batch 4: config 4 re-profiled at HEAD (trace + FETCH/WRITE + SQ/TCC of k_svd_topk /
# k_svd_merge) and its bench line with the per-pair reconstruction cpu_baseline; then
# experiment 1 (config-2 user side: LARGE block scorer against two half-universe chunks).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
bash profiles/scripts/r04_prof.sh r04_svd_c4 --mode svd || { echo "svd profile failed"; exit 1; }
timeout -k 10 300 python bench.py --mode svd > gpurun_out/r04b4_svd.json 2> gpurun_out/r04b4_svd.err || { tail -20 gpurun_out/r04b4_svd.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r04b4_svd.json'));print('svd', round(d['ms_per_step'],3), d['value'], d['roofline'], d['cpu_baseline'])"
bash profiles/scripts/r04_exp1.sh
