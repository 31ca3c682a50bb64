#!/bin/bash
# Round 3: norm-pruned SVD top-k -- GPU tests (pruned == dense == numpy), then config 4 with the
# dense headline and the pruned line.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_svd.py > gpurun_out/e26_tests.log 2>&1 || { tail -40 gpurun_out/e26_tests.log; exit 1; }
tail -3 gpurun_out/e26_tests.log
timeout -k 10 900 python -u bench.py --mode svd --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/e26_c4.json 2> gpurun_out/e26_c4.err || { tail -20 gpurun_out/e26_c4.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/e26_c4.json'));print(round(d['ms_per_step'],3), d['roofline']['kernel_ms'], d['parity'], d['pruned_topk'])"
