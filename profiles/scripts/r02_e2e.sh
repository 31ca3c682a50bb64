#!/bin/bash
# Round 2: GPU suite, then similarity.main end to end at config 1 (Yelp-sized) and config 2.
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=${TMPDIR:-/tmp}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r02_gputest.log 2>&1 || { tail -40 gpurun_out/r02_gputest.log; exit 1; }
tail -2 gpurun_out/r02_gputest.log
timeout -k 10 400 python bench.py --mode e2e --config yelp > gpurun_out/r02_e2e_yelp.json 2> gpurun_out/r02_e2e_yelp.err || { tail -30 gpurun_out/r02_e2e_yelp.err; exit 1; }
cat gpurun_out/r02_e2e_yelp.json
timeout -k 10 600 python bench.py --mode e2e --config c2 > gpurun_out/r02_e2e_c2.json 2> gpurun_out/r02_e2e_c2.err || { tail -30 gpurun_out/r02_e2e_c2.err; exit 1; }
cat gpurun_out/r02_e2e_c2.json
