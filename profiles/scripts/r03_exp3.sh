#!/bin/bash
# Round 3: split-scorer changes (prefetched batch metadata, fused offset scan, 2 atomics per slice)
# the fused offset scan in the large scorer, and the short-row scorer's thread-owned scan (A/B: libblp_x1.so) -- parity, config 2 / 5 timing, then a config-5
# rocprof pass set (trace + FETCH + WRITE + SQ/TCC counters) -> gpurun_out/r03_c5_v1*.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_similarity.py tests/test_gpu_headline.py tests/test_gpu_ingest.py -x -q --timeout 200 --timeout-method thread > gpurun_out/e3_tests.log 2>&1 || { tail -30 gpurun_out/e3_tests.log; exit 1; }
tail -2 gpurun_out/e3_tests.log
q() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/e3_$n.json 2> gpurun_out/e3_$n.err || { tail -20 gpurun_out/e3_$n.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/e3_$n.json'));print('$n', round(d['ms_per_step'],3), {k:(round(v['score_ms'],3),round(v['group_ms'],3)) for k,v in d.get('kernels_ms',{}).items()}, d['roofline'].get('kernel_ms'), (d.get('parity') or {}).get('ok'))"
}
L=$R/bipartite-link-prediction_amd/blp
q c2 || exit 1
BLP_LIB=$L/libblp_x1.so q c2_x1 --no-parity || exit 1
q c2_b --no-parity || exit 1
BLP_LIB=$L/libblp_x1.so q c2_x1_b --no-parity || exit 1
q c5 --mode sharded --config c5 --steps 3 --warmup 1 --no-parity || exit 1
bash profiles/scripts/r02_prof.sh r03_c5_v1 --mode sharded --config c5 --steps 2 > gpurun_out/e3_prof.log 2>&1 || { tail -20 gpurun_out/e3_prof.log; exit 1; }
grep -A22 "k_score_split" gpurun_out/r03_c5_v1_pmc.txt | head -50
head -12 gpurun_out/r03_c5_v1.md
