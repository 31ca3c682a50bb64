#!/bin/bash
# Round 5 call G: profile B (config 5's business pass alone, config 3's top-k step with the
# per-wave selection), then the config-3, config-4 and config-5 bench lines at HEAD (each line's
# traffic_source is the newest profile of its kernel).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
for i in 1 2; do
  BLP_E2E_REFDEBUG=1 BLP_GRAPH_PROF=1 BLP_SLOW_HIP_MS=3 timeout -k 10 300 python bench.py --mode e2e --config c2 > gpurun_out/r05g_e2e_$i.json 2> gpurun_out/r05g_e2e_$i.err || { tail -20 gpurun_out/r05g_e2e_$i.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r05g_e2e_$i.json').read().strip().splitlines()[-1]);print('e2e', round(d['e2e_s'],4), {k: round(v,4) for k,v in d['phases_s'].items()}, d['ok'])"
  grep refdebug gpurun_out/r05g_e2e_$i.err
done
bash profiles/scripts/r05_profB.sh || exit 1
head -8 gpurun_out/r05_topk_v1.md
timeout -k 10 600 python bench.py --mode topk > gpurun_out/r05g_topk.json 2> gpurun_out/r05g_topk.err || { tail -20 gpurun_out/r05g_topk.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r05g_topk.json'));print('c3', round(d['ms_per_step'],3), d['value'], d.get('parity'), d['roofline'])"
timeout -k 10 300 python bench.py --mode svd > gpurun_out/r05g_svd.json 2> gpurun_out/r05g_svd.err || { tail -20 gpurun_out/r05g_svd.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r05g_svd.json'));print('c4', round(d['ms_per_step'],3), d['value'], d.get('parity'), d['roofline'])"
timeout -k 10 900 python -u bench.py --mode sharded --config c5 --steps 3 --warmup 1 > gpurun_out/r05g_c5.json 2> gpurun_out/r05g_c5.err || { tail -20 gpurun_out/r05g_c5.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r05g_c5.json').read().strip().splitlines()[-1]);print('c5', round(d['ms_per_step'],3), d['value'], d.get('parity'), d['roofline'])"
