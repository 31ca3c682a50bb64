#!/bin/bash
# Round 6, profile call 1: the config-2 bench at HEAD (wedge-set business pass) -- kernel trace +
# stats, FETCH_SIZE / WRITE_SIZE, SQ and TCC passes -> gpurun_out/r06_v1_bench.{md,json}, _pmc.txt;
# then similarity.main at config 2 three times (stage clocks).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
bash profiles/scripts/r06_prof.sh r06_v1_bench 300 --steps 10 || exit 1
for i in 1 2 3; do
  BLP_GRAPH_PROF=1 timeout -k 10 300 python bench.py --mode e2e --config c2 > gpurun_out/r06p1_e2e_$i.json 2> gpurun_out/r06p1_e2e_$i.err || { tail -20 gpurun_out/r06p1_e2e_$i.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r06p1_e2e_$i.json').read().strip().splitlines()[-1]);print('e2e', round(d['e2e_s'],4), d['ok'], {k: round(v, 4) for k, v in d['phases_s'].items() if v > 0.003})"
  grep "device_parse" gpurun_out/r06p1_e2e_$i.err
done
