#!/bin/bash
# Round 6, final check 8 at HEAD (after the upload reorder): the whole GPU suite, smoke(), the default bench line (full
# parity + CPU baseline), similarity.main at configs 2 (twice) and 1, and the driver's N > 1
# launch path rehearsed with two ranks on the box's one GPU (BLP_DEVICE=0; RCCL refuses two
# ranks on one device, so the exchange reports that error and the headline line stands).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rs > gpurun_out/r06fin8_gputest.log 2>&1 || { tail -60 gpurun_out/r06fin8_gputest.log; exit 1; }
tail -3 gpurun_out/r06fin8_gputest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06fin8_smoke.log 2>&1 || { tail -20 gpurun_out/r06fin8_smoke.log; exit 1; }
tail -1 gpurun_out/r06fin8_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r06fin8_bench.json 2> gpurun_out/r06fin8_bench.err || { tail -20 gpurun_out/r06fin8_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r06fin8_bench.json'));print('bench', round(d['ms_per_step'],4), d['value'], d['kernels_ms'], d['parity']['ok'], d['roofline']['frac'], d['roofline'].get('frac_profile'), d['roofline'].get('frac_alone'), d['roofline_business']['frac'], d['cpu_baseline']['value'])"
for c in c2 c2 yelp; do
  timeout -k 10 300 python bench.py --mode e2e --config $c > gpurun_out/r06fin8_e2e_$c.json 2> gpurun_out/r06fin8_e2e_$c.err || { tail -20 gpurun_out/r06fin8_e2e_$c.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r06fin8_e2e_$c.json').read().strip().splitlines()[-1]);print('e2e $c', round(d['e2e_s'],4), d['ok'])"
done
BLP_DEVICE=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 2 --steps 5 --warmup 1 > gpurun_out/r06fin8_r2.json 2> gpurun_out/r06fin8_r2.err || { tail -30 gpurun_out/r06fin8_r2.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r06fin8_r2.json').read().strip().splitlines()[-1]);print('r2', d['n_gpus'], round(d['ms_per_step'],4), d['value'], (d.get('parity') or {}).get('ok'), (d.get('exchange') or {}).get('error'))"
