#!/bin/bash
# Round 6, A/B 3, alternating on one box: (1) similarity.main at config 2 with the 16 MiB staging
# ring allocated first by the prewarm (stage clocks); (2) the config-2 step, the default build
# against the header-prefetch build (pf) with fewer short-row workgroups per CU (BLP_SHORT_WGS).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
for i in 1 2 3; do
  BLP_GRAPH_PROF=1 timeout -k 10 300 python bench.py --mode e2e --config c2 > gpurun_out/r06ab3_e2e_$i.json 2> gpurun_out/r06ab3_e2e_$i.err || { tail -20 gpurun_out/r06ab3_e2e_$i.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r06ab3_e2e_$i.json').read().strip().splitlines()[-1]);print('e2e', round(d['e2e_s'],4), d['ok'], {k: round(v, 4) for k, v in d['phases_s'].items() if v > 0.003})"
  grep "device_parse" gpurun_out/r06ab3_e2e_$i.err
done
L=$R/bipartite-link-prediction_amd/blp
for round in 1 2; do
  for v in def:0 pf:6 pf:5 pf:4 def:6; do
    name=${v%%:*}; w=${v##*:}
    lib=$L/libblp.so
    [ $name != def ] && lib=$L/libblp_$name.so
    env=""
    [ $w != 0 ] && env="BLP_SHORT_WGS=$w"
    env $env BLP_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-exchange --no-parity > gpurun_out/r06ab3_${name}_${w}_$round.json 2> gpurun_out/r06ab3_${name}_${w}_$round.err || { tail -20 gpurun_out/r06ab3_${name}_${w}_$round.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r06ab3_${name}_${w}_$round.json'));print('$name', $w, $round, round(d['ms_per_step'],4), {k: {kk: round(vv, 4) for kk, vv in x.items()} for k, x in d['kernels_ms'].items()})"
  done
done
