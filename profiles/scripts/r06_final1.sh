#!/bin/bash
# Round 6, final check 1 at HEAD: the whole GPU suite, smoke(), the default bench line (full
# parity + CPU baseline), config 3, similarity.main at configs 2 and 1 (Yelp-sized).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rs > gpurun_out/r06fin1_gputest.log 2>&1 || { tail -60 gpurun_out/r06fin1_gputest.log; exit 1; }
tail -3 gpurun_out/r06fin1_gputest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06fin1_smoke.log 2>&1 || { tail -20 gpurun_out/r06fin1_smoke.log; exit 1; }
tail -1 gpurun_out/r06fin1_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r06fin1_bench.json 2> gpurun_out/r06fin1_bench.err || { tail -20 gpurun_out/r06fin1_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r06fin1_bench.json'));print('bench', round(d['ms_per_step'],4), d['value'], d['kernels_ms'], d['parity']['ok'], d['roofline']['frac'], d['roofline'].get('frac_profile'), d['roofline_business']['frac'], d['cpu_baseline']['value'])"
timeout -k 10 600 python bench.py --mode topk > gpurun_out/r06fin1_topk.json 2> gpurun_out/r06fin1_topk.err || { tail -20 gpurun_out/r06fin1_topk.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r06fin1_topk.json').read().strip().splitlines()[-1]);print('c3', round(d['ms_per_step'],3), d.get('parity', {}).get('jaccard_exact'))"
for c in c2 c2 yelp; do
  timeout -k 10 300 python bench.py --mode e2e --config $c > gpurun_out/r06fin1_e2e_$c.json 2> gpurun_out/r06fin1_e2e_$c.err || { tail -20 gpurun_out/r06fin1_e2e_$c.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r06fin1_e2e_$c.json').read().strip().splitlines()[-1]);print('e2e $c', round(d['e2e_s'],4), d['ok'])"
done
