#!/bin/bash
# Round 4, check 3: per-node two-hop statistics on the device (node2.hip) -- the scorer and
# wedge-row tests, device-side score-text formatting (repr.hip), the config-2 bench, and config 2 end to end with batch-create stage times.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_similarity.py tests/test_gpu_ingest.py tests/test_gpu_headline.py tests/test_gpu_hop3.py tests/test_gpu_debug.py tests/test_gpu_atsize.py tests/test_repr.py -m gpu -x -q --timeout 300 --timeout-method thread -rs > gpurun_out/r04c3_gputest.log 2>&1 || { tail -60 gpurun_out/r04c3_gputest.log; exit 1; }
tail -3 gpurun_out/r04c3_gputest.log
timeout -k 10 300 python bench.py > gpurun_out/r04c3_bench.json 2> gpurun_out/r04c3_bench.err || { tail -20 gpurun_out/r04c3_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r04c3_bench.json'));print('bench', round(d['ms_per_step'],3), d['value'], d['kernels_ms'], d['parity']['ok'], d['setup_s'])"
BLP_CREATE_PROF=1 BLP_GRAPH_PROF=1 timeout -k 10 300 python bench.py --mode e2e --config c2 > gpurun_out/r04c3_e2e.json 2> gpurun_out/r04c3_e2e.err || { tail -20 gpurun_out/r04c3_e2e.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r04c3_e2e.json').read().strip().splitlines()[-1]);print('e2e', d['e2e_s'], d['phases_s'], d['graph_phase_detail_s'], d['ok'])"
grep -E "blp_batch_create|graph_finish" gpurun_out/r04c3_e2e.err | tail -24
