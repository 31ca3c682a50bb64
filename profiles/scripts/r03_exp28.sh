#!/bin/bash
# Round 3: config 5 with a 20x larger at-scale parity sample (1,000 user + 1,000 business
# sources on the full 1B-edge graph).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 1100 python -u bench.py --mode sharded --config c5 --steps 3 --warmup 1 --no-cpu-baseline --parity-sources 1000 > gpurun_out/e28_c5_parity1000.json 2> gpurun_out/e28_c5_parity1000.err || { tail -20 gpurun_out/e28_c5_parity1000.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/e28_c5_parity1000.json'));print('c5', round(d['ms_per_step'],3), d['parity'])"
