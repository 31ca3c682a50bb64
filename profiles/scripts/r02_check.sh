#!/bin/bash
# Round-2 GPU check: the -m gpu suite, smoke(), and the default bench (config 2).
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r02_gputest.log 2>&1 || { tail -30 gpurun_out/r02_gputest.log; exit 1; }
tail -3 gpurun_out/r02_gputest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_smoke.log 2>&1 || { cat gpurun_out/r02_smoke.log; exit 1; }
cat gpurun_out/r02_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r02_bench.json 2> gpurun_out/r02_bench.err || { tail -30 gpurun_out/r02_bench.err; exit 1; }
cat gpurun_out/r02_bench.json
