#!/bin/bash
# Round 6, profile call 2: config 5's user pass at HEAD (trace, FETCH_SIZE, WRITE_SIZE, SQ and TCC
# passes; r06_prof.sh), then the config-5 bench line (both passes, parity on 50 + 50 sources).
# First the new split-scorer escape-path knob tests.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_similarity.py -k kernel_paths_vs_oracle -x -q --timeout 300 --timeout-method thread > gpurun_out/r06pc2_tests.log 2>&1 || { tail -30 gpurun_out/r06pc2_tests.log; exit 1; }
tail -1 gpurun_out/r06pc2_tests.log
bash profiles/scripts/r06_prof.sh r06_c5_user 300 --mode sharded --config c5 --sides user --steps 2 || exit 1
cd $R
timeout -k 10 600 python -u bench.py --mode sharded --config c5 --steps 3 --warmup 1 > gpurun_out/r06pc2_c5.json 2> gpurun_out/r06pc2_c5.err || { tail -20 gpurun_out/r06pc2_c5.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r06pc2_c5.json').read().strip().splitlines()[-1]);r=d['roofline'];print('c5', round(d['ms_per_step'],2), d['value'], d.get('parity', {}).get('ok'), round(r['kernel_ms'],2), round(r['frac'],4), r.get('traffic_source'))"
