#!/bin/bash
# Round 3 experiments: config-3 16-byte row tails (A/B), the config-2 step decomposed (user mask,
# one side alone), then config 5 (RCCL exchange at world 1 + the new 1B-edge oracle parity block).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
L=$R/bipartite-link-prediction_amd/blp
q() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity "$@" > gpurun_out/e1_$n.json 2> gpurun_out/e1_$n.err || { tail -20 gpurun_out/e1_$n.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/e1_$n.json'));print('$n', round(d['ms_per_step'],3), {k:(round(v['score_ms'],3),round(v['group_ms'],3)) for k,v in d.get('kernels_ms',{}).items()}, d['roofline'].get('kernel_ms'))"
}
q topk_base --mode topk --steps 5 --warmup 1 || exit 1
BLP_LIB=$L/libblp_t16.so q topk_t16 --mode topk --steps 5 --warmup 1 || exit 1
q topk_base2 --mode topk --steps 5 --warmup 1 || exit 1
q c2 || exit 1
q c2_mask3 --user-mask 3 || exit 1
q c2_mask1 --user-mask 1 || exit 1
q c2_user --sides user || exit 1
q c2_bus --sides business || exit 1
timeout -k 10 900 python -u bench.py --mode sharded --config c5 --steps 3 --warmup 1 > gpurun_out/e1_c5.json 2> gpurun_out/e1_c5.err || { tail -30 gpurun_out/e1_c5.err; exit 1; }
cat gpurun_out/e1_c5.json
