#!/bin/bash
# Round 3: wedge-row bitmaps for hop-3 (tests, then config-2 setup A/B), run-ordered item writes (A/B), config-2 sides alone
# (full chip each), and the config-3 top-k trace + counters.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_hop3.py -x -q --timeout 120 --timeout-method thread > gpurun_out/e10_hop3.log 2>&1 || { tail -30 gpurun_out/e10_hop3.log; exit 1; }
tail -2 gpurun_out/e10_hop3.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_similarity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/e10_sim.log 2>&1 || { tail -30 gpurun_out/e10_sim.log; exit 1; }
tail -2 gpurun_out/e10_sim.log
q() {  # name, args...
  local n=$1; shift
  timeout -k 10 600 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/e10_$n.json 2> gpurun_out/e10_$n.err || { tail -20 gpurun_out/e10_$n.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/e10_$n.json'));print('$n', round(d['ms_per_step'],3), d.get('kernels_ms'), d.get('setup_s'))"
}
q c2 --steps 20 --warmup 3 || exit 1
BLP_HOP3_NO_WBM=1 q c2_nowbm --steps 20 --warmup 3 --no-parity || exit 1
BLP_ITEM_SCATTER=1 q c2_scatter --steps 20 --warmup 3 --no-parity || exit 1
BLP_GROUP_BUCKETS=1 q c2_buckets --steps 20 --warmup 3 --no-parity || exit 1
q c2_user --steps 20 --warmup 3 --no-parity --sides user || exit 1
q c2_bus --steps 20 --warmup 3 --no-parity --sides business || exit 1
bash profiles/scripts/r03_prof.sh r03_topk_v3 --mode topk > gpurun_out/e10_prof.log 2>&1 || { tail -20 gpurun_out/e10_prof.log; exit 1; }
head -14 gpurun_out/r03_topk_v3.md | cut -c1-220
grep -B1 -A18 "k_topk" gpurun_out/r03_topk_v3_pmc.txt | head -42
