#!/bin/bash
# Round 5, final check 6 at HEAD (after the last default change): the whole GPU suite, smoke(), the
# default bench line, config-2 similarity.main twice, the config-3 line.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rs > gpurun_out/r05fin6_gputest.log 2>&1 || { tail -60 gpurun_out/r05fin6_gputest.log; exit 1; }
tail -3 gpurun_out/r05fin6_gputest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05fin6_smoke.log 2>&1 || { tail -20 gpurun_out/r05fin6_smoke.log; exit 1; }
tail -1 gpurun_out/r05fin6_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r05fin6_bench.json 2> gpurun_out/r05fin6_bench.err || { tail -20 gpurun_out/r05fin6_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r05fin6_bench.json'));print('bench', round(d['ms_per_step'],3), d['value'], d['kernels_ms'], d['parity']['ok'])"
for i in 1 2; do
  timeout -k 10 300 python bench.py --mode e2e --config c2 > gpurun_out/r05fin6_e2e_$i.json 2> gpurun_out/r05fin6_e2e_$i.err || { tail -20 gpurun_out/r05fin6_e2e_$i.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r05fin6_e2e_$i.json').read().strip().splitlines()[-1]);print('e2e', round(d['e2e_s'],4), d['ok'])"
done
timeout -k 10 600 python bench.py --mode topk > gpurun_out/r05fin6_topk.json 2> gpurun_out/r05fin6_topk.err || { tail -20 gpurun_out/r05fin6_topk.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r05fin6_topk.json').read().strip().splitlines()[-1]);print('c3', round(d['ms_per_step'],3), d.get('parity', {}).get('jaccard_exact'))"
