#!/bin/bash
# Round 6, check 4: wedge-set scorer with 2 pairs per thread (pp2 build) against the default
# (1 pair), alternating, at HEAD (run-grouped batches write no identity g_out); then the whole
# GPU suite, smoke() and the default bench line with full parity.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
L=$R/bipartite-link-prediction_amd/blp
for round in 1 2 3; do
  for v in def pp2; do
    lib=$L/libblp.so
    [ $v != def ] && lib=$L/libblp_$v.so
    BLP_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-exchange --no-parity > gpurun_out/r06c4_${v}_$round.json 2> gpurun_out/r06c4_${v}_$round.err || { tail -20 gpurun_out/r06c4_${v}_$round.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r06c4_${v}_$round.json'));print('$v', $round, round(d['ms_per_step'],4), {k: {kk: round(vv, 4) for kk, vv in x.items()} for k, x in d['kernels_ms'].items()})"
  done
done
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rs > gpurun_out/r06c4_gputest.log 2>&1 || { tail -40 gpurun_out/r06c4_gputest.log; exit 1; }
tail -3 gpurun_out/r06c4_gputest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06c4_smoke.log 2>&1 || { tail -20 gpurun_out/r06c4_smoke.log; exit 1; }
tail -1 gpurun_out/r06c4_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r06c4_bench.json 2> gpurun_out/r06c4_bench.err || { tail -20 gpurun_out/r06c4_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r06c4_bench.json'));print('bench', round(d['ms_per_step'],4), d['value'], d['kernels_ms'], d['parity']['ok'], d['roofline']['frac'], d['roofline_business']['frac'])"
