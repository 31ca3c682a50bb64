#!/bin/bash
# Round 6, A/B 19, alternating on one box: config 2 with the block scorer's VGPRs capped so that
# the wedge-set launch's waves (24 VGPRs, no LDS) can co-reside with the user scorer's workgroups
# and run in its latency stalls: amdgpu_num_vgpr(52) -> 104 registers (libblp_v52.so: 96 per
# SIMD lane left, four wedge-set waves), (56) -> 112 (libblp_v56.so: two), against no cap
# (libblp.so: 128 registers, nothing co-resides). The first arm of each cap checks parity.
# Result (r06_ab19.txt): the launches co-reside (business in-step 1.1-1.5 -> 0.36-0.48 ms) but the
# capped scorer alone slows 1.465 -> 1.58-1.60 ms; steps 1.674-1.713 against 1.662-1.718. The
# experiment macro (BLP_PKO_VGPR: amdgpu_num_vgpr, doubled on gfx950) was removed.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
L=$R/bipartite-link-prediction_amd/blp
run() {  # name lib [extra]
  BLP_LIB=$L/$2 timeout -k 10 300 python bench.py --no-cpu-baseline --no-exchange ${3:---no-parity} > gpurun_out/r06ab19_$1.json 2> gpurun_out/r06ab19_$1.err || { tail -20 gpurun_out/r06ab19_$1.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r06ab19_$1.json'));r=d['roofline'];print('$1', round(d['ms_per_step'],4), (d.get('parity') or {}).get('ok'), {k: {kk: round(vv, 4) for kk, vv in x.items()} for k, x in d['kernels_ms'].items()}, 'alone', round(r.get('kernel_alone_ms') or 0, 4), round(d['roofline_business'].get('kernel_alone_ms') or 0, 4))"
}
run v52_0 libblp_v52.so --steps=20 && run v56_0 libblp_v56.so --steps=20 || exit 1
for round in 1 2 3; do
  run base_$round libblp.so && run v52_$round libblp_v52.so && run v56_$round libblp_v56.so || exit 1
done
