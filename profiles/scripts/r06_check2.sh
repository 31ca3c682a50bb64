#!/bin/bash
# Round 6, check 2 (after the scorer-variant removal): the whole GPU suite, smoke(), the default
# bench line, config-2 similarity.main twice with the parse stage clocks.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rs > gpurun_out/r06c2_gputest.log 2>&1 || { tail -60 gpurun_out/r06c2_gputest.log; exit 1; }
tail -3 gpurun_out/r06c2_gputest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06c2_smoke.log 2>&1 || { tail -20 gpurun_out/r06c2_smoke.log; exit 1; }
tail -1 gpurun_out/r06c2_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r06c2_bench.json 2> gpurun_out/r06c2_bench.err || { tail -20 gpurun_out/r06c2_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r06c2_bench.json'));print('bench', round(d['ms_per_step'],3), d['value'], d['kernels_ms'], d['parity']['ok'])"
for i in 1 2; do
  BLP_GRAPH_PROF=1 timeout -k 10 300 python bench.py --mode e2e --config c2 > gpurun_out/r06c2_e2e_$i.json 2> gpurun_out/r06c2_e2e_$i.err || { tail -20 gpurun_out/r06c2_e2e_$i.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r06c2_e2e_$i.json').read().strip().splitlines()[-1]);print('e2e', round(d['e2e_s'],4), d['ok'], d['phases_s'])"
  grep device_parse gpurun_out/r06c2_e2e_$i.err
done
timeout -k 10 600 python bench.py --mode topk > gpurun_out/r06c2_topk.json 2> gpurun_out/r06c2_topk.err || { tail -20 gpurun_out/r06c2_topk.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r06c2_topk.json').read().strip().splitlines()[-1]);print('c3', round(d['ms_per_step'],3), d.get('parity', {}))"
BLP_LIB=$R/bipartite-link-prediction_amd/blp/libblp_prof.so SWEEP_PROF=1 SWEEP_STEPS=3 timeout -k 10 300 python profiles/sweep.py > gpurun_out/r06c2_prof_sweep.txt 2>&1 || { tail -20 gpurun_out/r06c2_prof_sweep.txt; exit 1; }
cat gpurun_out/r06c2_prof_sweep.txt | tail -4
