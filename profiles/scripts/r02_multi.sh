#!/bin/bash
# Round 2: bench.py --gpus 2 self-launch (two ranks sharing the one GPU: BLP_DEVICE=0), then the
# config-5 row-block sharded ingest + device CSR build + scoring at 1 GPU.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
BLP_DEVICE=0 timeout -k 10 400 python bench.py --gpus 2 --no-cpu-baseline --steps 10 > gpurun_out/r02_gpus2.json 2> gpurun_out/r02_gpus2.err || { tail -30 gpurun_out/r02_gpus2.err; exit 1; }
cat gpurun_out/r02_gpus2.json
timeout -k 10 900 python -u bench.py --mode sharded --config c5 --steps 5 --warmup 1 > gpurun_out/r02_c5.json 2> gpurun_out/r02_c5.err || { tail -30 gpurun_out/r02_c5.err; exit 1; }
cat gpurun_out/r02_c5.json
