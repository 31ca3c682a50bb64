#!/bin/bash
# Round 3: wedge rows for every node whose members' rows are <= 64 ids (hub nodes filled by items),
# used by the chunk-parallel and hash-set scorers -- ingest / similarity / hop-3 tests, then
# config 5 (parity) with and without them, and config 2 (unchanged path, parity).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ingest.py tests/test_gpu_similarity.py tests/test_gpu_hop3.py -x -q --timeout 120 --timeout-method thread > gpurun_out/e20_tests.log 2>&1 || { tail -30 gpurun_out/e20_tests.log; exit 1; }
tail -2 gpurun_out/e20_tests.log
q() {  # name, args...
  local n=$1; shift
  timeout -k 10 900 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/e20_$n.json 2> gpurun_out/e20_$n.err || { tail -20 gpurun_out/e20_$n.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/e20_$n.json'));print('$n', round(d['ms_per_step'],3), d['roofline'].get('kernel_ms'), (d.get('parity') or {}).get('ok'), d.get('exchange', {}).get('device_csr_phases_s'), d.get('kernels_ms'))"
}
q c5 --mode sharded --config c5 --steps 3 --warmup 1 || exit 1
q c5_bus --mode sharded --config c5 --steps 3 --warmup 1 --no-parity --sides business || exit 1
BLP_NO_WEDGE=1 q c5_bus_nowedge --mode sharded --config c5 --steps 3 --warmup 1 --no-parity --sides business || exit 1
q c2 --steps 20 --warmup 3 || exit 1
