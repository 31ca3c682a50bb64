#!/bin/bash
# Round 3: full parity at scale -- config 3 lists of ALL 10K users against the C oracle, config 4
# lists of ALL 10K users against fp64 numpy (dense and pruned paths equal).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py --mode topk --steps 3 --warmup 1 --no-cpu-baseline --topk-parity-users 0 > gpurun_out/e27_topk_full.json 2> gpurun_out/e27_topk_full.err || { tail -20 gpurun_out/e27_topk_full.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/e27_topk_full.json'));print('topk', round(d['ms_per_step'],3), d['parity'])"
timeout -k 10 900 python -u bench.py --mode svd --steps 3 --warmup 1 --no-cpu-baseline --svd-parity-users 0 > gpurun_out/e27_svd_full.json 2> gpurun_out/e27_svd_full.err || { tail -20 gpurun_out/e27_svd_full.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/e27_svd_full.json'));print('svd', round(d['ms_per_step'],3), d['parity'], d['pruned_topk']['lists_equal_dense'])"
