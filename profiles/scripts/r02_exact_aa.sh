#!/bin/bash
# Round 2: exact Adamic-Adar sums -- the -m gpu suite, smoke(), the default bench (config 2)
# and the config-3 top-k bench (AA keys now exact doubles).
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r02_gputest.log 2>&1 || { tail -40 gpurun_out/r02_gputest.log; exit 1; }
tail -3 gpurun_out/r02_gputest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_smoke.log 2>&1 || { cat gpurun_out/r02_smoke.log; exit 1; }
cat gpurun_out/r02_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r02_bench.json 2> gpurun_out/r02_bench.err || { tail -30 gpurun_out/r02_bench.err; exit 1; }
cat gpurun_out/r02_bench.json
timeout -k 10 400 python bench.py --mode topk > gpurun_out/r02_topk.json 2> gpurun_out/r02_topk.err || { tail -30 gpurun_out/r02_topk.err; exit 1; }
cat gpurun_out/r02_topk.json
