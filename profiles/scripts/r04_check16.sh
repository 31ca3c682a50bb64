#!/bin/bash
# device graph.txt parse tests first, then the whole final check (r04_final.sh)
set -o pipefail
mkdir -p gpurun_out/c15
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ingest.py \
  -k "device_parse or load_edge_list" > gpurun_out/c15/t1.txt 2>&1 || { tail -40 gpurun_out/c15/t1.txt; exit 1; }
tail -3 gpurun_out/c15/t1.txt
bash profiles/scripts/r04_final.sh
