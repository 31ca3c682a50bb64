#!/bin/bash
# Round 5 A/B 7: the large scorer's one-scan segment offsets (libblp_exp5.so, -DBLP_SEGOFF=1)
# against the default, alternating; config 2 end to end twice (pooled streams, one upload); then
# the config-5 profile at HEAD (r05_c5: trace + FETCH/WRITE + SQ/TCC of both passes).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
run() {  # name, env...
  local n=$1
  shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity --no-exchange --steps 30 > gpurun_out/r05ab7_$n.json 2> gpurun_out/r05ab7_$n.err || { tail -20 gpurun_out/r05ab7_$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r05ab7_$n.json'));print('$n', round(d['ms_per_step'],3), {k:{a:round(b,3) for a,b in v.items()} for k,v in d['kernels_ms'].items()}, d['including_batch_create']['batch_create_s'])"
}
for i in 1 2 3; do
  run def_$i
  run segoff_$i BLP_LIB=$R/bipartite-link-prediction_amd/blp/libblp_exp5.so
done
for i in 1 2; do
  BLP_CREATE_PROF=1 BLP_GRAPH_PROF=1 timeout -k 10 300 python bench.py --mode e2e --config c2 > gpurun_out/r05ab7_e2e_$i.json 2> gpurun_out/r05ab7_e2e_$i.err || { tail -20 gpurun_out/r05ab7_e2e_$i.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r05ab7_e2e_$i.json').read().strip().splitlines()[-1]);print('e2e', round(d['e2e_s'],4), {k: round(v,4) for k,v in d['phases_s'].items()}, d['graph_phase_detail_s'], d['ok'])"
done
bash profiles/scripts/r05_prof.sh r05_c5 300 --mode sharded --config c5 --steps 3 || exit 1
