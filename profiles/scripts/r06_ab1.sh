#!/bin/bash
# Round 6, A/B 1, alternating on one box.
# Config-2 step: the default build against experiment builds -- rbo: k_score_short's wedge build
# reads each bitmap word before OR-ing it (-DBLP_SHORT_RBO=1); pf: k_score_short stages the next
# source's record in LDS (-DBLP_SHORT_PF=1); pfrbo: both; quad: rc_scan's packed AA hits summed
# within a quad before the LDS atomics (-DBLP_RC_QUAD=1). Round 1 with full 15.09M-score parity.
# Config 3: k_topk's arguments through a pointer (default) against by value (tkbv, -DBLP_TK_ARGPTR=0).
# (as run: round 2 of config 3 carried --topk-parity-users 0, every user's lists checked.)
# similarity.main at config 2: the graph.txt staging ring with 16 and 8 readers (stage clocks).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
L=$R/bipartite-link-prediction_amd/blp
for round in 1 2 3; do
  extra="--no-cpu-baseline --no-exchange"
  [ $round -gt 1 ] && extra="$extra --no-parity"
  for v in def rbo pf pfrbo quad; do
    lib=$L/libblp.so
    [ $v != def ] && lib=$L/libblp_$v.so
    BLP_LIB=$lib timeout -k 10 300 python bench.py $extra > gpurun_out/r06ab1_${v}_$round.json 2> gpurun_out/r06ab1_${v}_$round.err || { tail -20 gpurun_out/r06ab1_${v}_$round.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r06ab1_${v}_$round.json'));print('$v', $round, round(d['ms_per_step'],4), {k: {kk: round(vv, 4) for kk, vv in x.items()} for k, x in d['kernels_ms'].items()}, d.get('parity', {}).get('ok'))"
  done
done
for round in 1 2; do
  for v in def tkbv; do
    lib=$L/libblp.so
    [ $v != def ] && lib=$L/libblp_$v.so
    extra=""
    BLP_LIB=$lib timeout -k 10 600 python bench.py --mode topk $extra > gpurun_out/r06ab1_c3_${v}_$round.json 2> gpurun_out/r06ab1_c3_${v}_$round.err || { tail -20 gpurun_out/r06ab1_c3_${v}_$round.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/r06ab1_c3_${v}_$round.json').read().strip().splitlines()[-1]);print('c3 $v', $round, round(d['ms_per_step'],4), d.get('parity', {}).get('jaccard_exact'))"
  done
done
for rd in 16 8 16 8; do
  BLP_PARSE_READERS=$rd BLP_GRAPH_PROF=1 timeout -k 10 300 python bench.py --mode e2e --config c2 > gpurun_out/r06ab1_e2e_r$rd.json 2> gpurun_out/r06ab1_e2e_r$rd.err || { tail -20 gpurun_out/r06ab1_e2e_r$rd.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r06ab1_e2e_r$rd.json').read().strip().splitlines()[-1]);print('e2e readers $rd', round(d['e2e_s'],4), d['ok'], round(d['phases_s']['graph'], 4))"
  grep "device_parse" gpurun_out/r06ab1_e2e_r$rd.err
done
