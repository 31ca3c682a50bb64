#!/bin/bash
# Round 4, check 4: device repr test, the config-2 bench and end to end (graph / create stage
# times), then config 4 re-profiled (trace + FETCH/WRITE + SQ/TCC) with its bench line, then
# experiment 1 (config-2 user side: LARGE block scorer against two half-universe chunks).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_repr.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04c4_gputest.log 2>&1 || { tail -30 gpurun_out/r04c4_gputest.log; exit 1; }
tail -1 gpurun_out/r04c4_gputest.log
timeout -k 10 300 python bench.py > gpurun_out/r04c4_bench.json 2> gpurun_out/r04c4_bench.err || { tail -20 gpurun_out/r04c4_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r04c4_bench.json'));print('bench', round(d['ms_per_step'],3), d['value'], d['kernels_ms'], d['parity']['ok'], d['setup_s'])"
BLP_CREATE_PROF=1 BLP_GRAPH_PROF=1 timeout -k 10 300 python bench.py --mode e2e --config c2 > gpurun_out/r04c4_e2e.json 2> gpurun_out/r04c4_e2e.err || { tail -20 gpurun_out/r04c4_e2e.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r04c4_e2e.json').read().strip().splitlines()[-1]);print('e2e', d['e2e_s'], d['phases_s'], d['graph_phase_detail_s'], d['ok'])"
grep -E "blp_batch_create|graph_finish" gpurun_out/r04c4_e2e.err | tail -24
bash profiles/scripts/r04_prof.sh r04_svd_c4 --mode svd || { echo "svd profile failed"; exit 1; }
timeout -k 10 300 python bench.py --mode svd > gpurun_out/r04c4_svd.json 2> gpurun_out/r04c4_svd.err || { tail -20 gpurun_out/r04c4_svd.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r04c4_svd.json'));print('svd', round(d['ms_per_step'],3), d['value'], d['roofline'], d['cpu_baseline'])"
bash profiles/scripts/r04_exp1.sh
