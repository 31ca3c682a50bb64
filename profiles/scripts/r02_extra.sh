#!/bin/bash
# Business pass with Adamic-Adar (fix_adamic), grouping unroll A/B, then config 5 at 1 GPU.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
timeout -k 10 300 python bench.py --fix-adamic --no-cpu-baseline > gpurun_out/r02x_fixaa.json 2> gpurun_out/r02x_fixaa.err || { tail -20 gpurun_out/r02x_fixaa.err; exit 1; }
tail -c 1500 gpurun_out/r02x_fixaa.json
for L in libblp.so libblp_gu8.so libblp.so libblp_gu8.so; do
  BLP_LIB=$R/bipartite-link-prediction_amd/blp/$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-parity > gpurun_out/gu.json 2>/dev/null || exit 1
  echo $L; cat gpurun_out/gu.json
done
timeout -k 10 900 python -u bench.py --mode sharded --config c5 --steps 5 --warmup 1 > gpurun_out/r02x_c5.json 2> gpurun_out/r02x_c5.err || { tail -30 gpurun_out/r02x_c5.err; exit 1; }
cat gpurun_out/r02x_c5.json
