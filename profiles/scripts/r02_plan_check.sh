#!/bin/bash
# batch-planning change: score-phase timing, GPU suite, quick config-2 bench
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python profiles/scripts/e2e_score_phases.py || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r02_gputest.log 2>&1 || { tail -40 gpurun_out/r02_gputest.log; exit 1; }
tail -2 gpurun_out/r02_gputest.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/q_bench.json 2> gpurun_out/q_bench.err || { tail -30 gpurun_out/q_bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/q_bench.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['setup_s'], d.get('parity', {}).get('ok'))"
