#!/bin/bash
# Round 3: config-5 user pass -- phase clocks of k_score_split (BLP_PROF experiment library).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
BLP_PROF_READ=1 BLP_LIB=$R/bipartite-link-prediction_amd/blp/libblp_prof.so timeout -k 10 900 python -u bench.py --no-cpu-baseline --mode sharded --config c5 --steps 2 --warmup 1 --no-parity --sides user > gpurun_out/e22_user_prof.json 2> gpurun_out/e22_user_prof.err || { tail -20 gpurun_out/e22_user_prof.err; exit 1; }
grep -a "prof\|plan" gpurun_out/e22_user_prof.err
python -c "import json;d=json.load(open('gpurun_out/e22_user_prof.json'));print(round(d['ms_per_step'],3), d['roofline'].get('kernel_ms'))"
