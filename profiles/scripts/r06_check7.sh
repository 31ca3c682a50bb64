#!/bin/bash
# Round 6, check 7: the knob matrix after tying the two-launch run grouping to the direct row
# lookup (BLP_VARIANT=2 with BLP_NO_YDIRECT / BLP_NO_RUN_FAST), the headline tests, and a config-2
# bench line with BLP_NO_YDIRECT=1 (gathered rows; full parity).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_similarity.py tests/test_gpu_headline.py -k "kernel_paths or headline or config2" -x -q --timeout 300 --timeout-method thread > gpurun_out/r06c7_tests.log 2>&1 || { tail -30 gpurun_out/r06c7_tests.log; exit 1; }
tail -1 gpurun_out/r06c7_tests.log
BLP_NO_YDIRECT=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-exchange > gpurun_out/r06c7_noyd.json 2> gpurun_out/r06c7_noyd.err || { tail -20 gpurun_out/r06c7_noyd.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r06c7_noyd.json'));r=d['roofline'];print('noyd', round(d['ms_per_step'],4), d['parity']['ok'], d['kernels_ms'], 'alone', r.get('kernel_alone_ms'))"
timeout -k 10 300 python bench.py --no-cpu-baseline --no-exchange > gpurun_out/r06c7_def.json 2> gpurun_out/r06c7_def.err || { tail -20 gpurun_out/r06c7_def.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r06c7_def.json'));r=d['roofline'];print('def', round(d['ms_per_step'],4), d['parity']['ok'], d['kernels_ms'], 'alone', r.get('kernel_alone_ms'))"
