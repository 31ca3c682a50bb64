#!/bin/bash
# wedge rows filled on the device: graph-phase timing, GPU suite, e2e config 2, quick bench
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python profiles/scripts/e2e_graph_phases.py || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r02_gputest.log 2>&1 || { tail -40 gpurun_out/r02_gputest.log; exit 1; }
tail -2 gpurun_out/r02_gputest.log
timeout -k 10 600 python bench.py --mode e2e --config c2 > gpurun_out/r02_e2e_c2.json 2> gpurun_out/r02_e2e_c2.err || { tail -30 gpurun_out/r02_e2e_c2.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r02_e2e_c2.json').read().strip().splitlines()[-1]); print(d['e2e_s'], d['phases_s'], d['ok'])"
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/q_bench.json 2> gpurun_out/q_bench.err || { tail -30 gpurun_out/q_bench.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/q_bench.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['setup_s'], d.get('parity', {}).get('ok'))"
