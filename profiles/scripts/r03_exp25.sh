#!/bin/bash
# Round 3: the C-ABI multi-GPU exchange (blp_multi_*, libblp's own RCCL communicator) -- GPU
# tests (world 1 host / device partials, two ranks on the one GPU), then config 5 through it.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ingest.py -k "multi_capi" -rs > gpurun_out/e25_tests.log 2>&1 || { tail -40 gpurun_out/e25_tests.log; exit 1; }
grep -a "PASS\|SKIP\|FAIL\|passed\|skipped" gpurun_out/e25_tests.log | tail -8
timeout -k 10 900 python -u bench.py --no-cpu-baseline --mode sharded --config c5 --steps 2 --warmup 1 --exchange capi > gpurun_out/e25_c5_capi.json 2> gpurun_out/e25_c5_capi.err || { tail -20 gpurun_out/e25_c5_capi.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/e25_c5_capi.json'));print(round(d['ms_per_step'],3), d['exchange'], d.get('parity',{}).get('ok'))"
