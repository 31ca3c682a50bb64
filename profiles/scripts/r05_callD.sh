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
BLP_LIB=$R/bipartite-link-prediction_amd/blp/libblp_debug.so timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_topk.py -k "wavesel or pruning" > gpurun_out/r05_topk_tests_debug.log 2>&1 || { tail -30 gpurun_out/r05_topk_tests_debug.log; exit 1; }
tail -3 gpurun_out/r05_topk_tests_debug.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_topk.py > gpurun_out/r05_topk_tests.log 2>&1 || { tail -30 gpurun_out/r05_topk_tests.log; exit 1; }
tail -3 gpurun_out/r05_topk_tests.log
for w in 0 1; do
  BLP_TK_WAVESEL=$w BLP_LIB=$R/bipartite-link-prediction_amd/blp/libblp_tkprof.so timeout -k 10 300 python profiles/scripts/topk_probe.py >> gpurun_out/r05_topk_phases.txt 2>&1 || { tail gpurun_out/r05_topk_phases.txt; exit 1; }
done
cat gpurun_out/r05_topk_phases.txt
BLP_LIB=$R/bipartite-link-prediction_amd/blp/libblp_tk512.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_topk.py tests/test_gpu_atsize.py -k "topk" > gpurun_out/r05_topk_tests_512.log 2>&1 || { tail -30 gpurun_out/r05_topk_tests_512.log; exit 1; }
tail -2 gpurun_out/r05_topk_tests_512.log
tk() {  # name, env...
  local n=$1
  shift
  env "$@" timeout -k 10 300 python bench.py --mode topk --steps 10 > gpurun_out/r05tk_$n.json 2> gpurun_out/r05tk_$n.err || { tail gpurun_out/r05tk_$n.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r05tk_$n.json').read().strip().splitlines()[-1]);print('$n', d['ms_per_step'], d.get('parity'))"
}
for i in 1 2; do
  tk def_$i
  tk wave_$i BLP_TK_WAVESEL=1
  tk nt512_$i BLP_LIB=$R/bipartite-link-prediction_amd/blp/libblp_tk512.so
  tk nt512w_$i BLP_LIB=$R/bipartite-link-prediction_amd/blp/libblp_tk512.so BLP_TK_WAVESEL=1
done
echo "call D done"
