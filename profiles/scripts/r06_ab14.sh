#!/bin/bash
# Round 6, A/B 14, alternating on one box: config 2 with the graph's score / group totals taken
# from the batches' own timers (libblp.so: two timing events per stream boundary instead of four)
# against HEAD before the change (libblp_prev.so). Then the timer tests.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
L=$R/bipartite-link-prediction_amd/blp
timeout -k 10 300 python -u -m pytest tests/test_gpu_similarity.py -k "totals_follow or repeat_is_deterministic" -x -q --timeout 120 --timeout-method thread > gpurun_out/r06ab14_tests.log 2>&1 || { tail -30 gpurun_out/r06ab14_tests.log; exit 1; }
tail -1 gpurun_out/r06ab14_tests.log
run() {  # name lib
  BLP_LIB=$L/$2 timeout -k 10 300 python bench.py --no-cpu-baseline --no-exchange --no-parity > gpurun_out/r06ab14_$1.json 2> gpurun_out/r06ab14_$1.err || { tail -20 gpurun_out/r06ab14_$1.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r06ab14_$1.json'));print('$1', round(d['ms_per_step'],4), {k: {kk: round(vv, 4) for kk, vv in x.items()} for k, x in d['kernels_ms'].items()})"
}
for round in 1 2 3 4; do
  run new_$round libblp.so && run prev_$round libblp_prev.so || exit 1
done
