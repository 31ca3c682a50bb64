#!/bin/bash
# Round 6, A/B 5, alternating on one box: the wedge-set scorer with blocked pair ranges and the
# user's row kept in registers (default build) against the grid-stride version (prev: HEAD before).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_similarity.py -k "wedge_set_path or kernel_paths" tests/test_gpu_debug.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06ab5_tests.log 2>&1 || { tail -40 gpurun_out/r06ab5_tests.log; exit 1; }
tail -2 gpurun_out/r06ab5_tests.log
L=$R/bipartite-link-prediction_amd/blp
for round in 1 2 3; do
  extra="--no-cpu-baseline --no-exchange"
  [ $round -gt 1 ] && extra="$extra --no-parity"
  for v in def prev; do
    lib=$L/libblp.so
    [ $v != def ] && lib=$L/libblp_$v.so
    BLP_LIB=$lib timeout -k 10 300 python bench.py $extra > gpurun_out/r06ab5_${v}_$round.json 2> gpurun_out/r06ab5_${v}_$round.err || { tail -20 gpurun_out/r06ab5_${v}_$round.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r06ab5_${v}_$round.json'));print('$v', $round, round(d['ms_per_step'],4), {k: {kk: round(vv, 4) for kk, vv in x.items()} for k, x in d['kernels_ms'].items()}, d.get('parity', {}).get('ok'))"
  done
done
