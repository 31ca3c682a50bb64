#!/bin/bash
# Round 5 A/B 5: the whole GPU suite; then config 2's business grouping -- rows carried by the
# scatter (default) against rows gathered by the write kernel (BLP_GROUP_GATHER=1) and the
# segment short-row scorer (BLP_SHORT_SEG=1) -- alternating; config 2 end to end twice.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 400 --timeout-method thread -rs > gpurun_out/r05ab5_gputest.log 2>&1 || { tail -80 gpurun_out/r05ab5_gputest.log; exit 1; }
tail -3 gpurun_out/r05ab5_gputest.log
grep "config5 1B" gpurun_out/r05ab5_gputest.log
run() {  # name, env...
  local n=$1
  shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity --no-exchange --steps 30 > gpurun_out/r05ab5_$n.json 2> gpurun_out/r05ab5_$n.err || { tail -20 gpurun_out/r05ab5_$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r05ab5_$n.json'));print('$n', round(d['ms_per_step'],3), {k:{a:round(b,3) for a,b in v.items()} for k,v in d['kernels_ms'].items()}, d['including_batch_create'])"
}
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r05ab5_parity.json 2> gpurun_out/r05ab5_parity.err || { tail -20 gpurun_out/r05ab5_parity.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r05ab5_parity.json'));print('parity bench', round(d['ms_per_step'],3), d['kernels_ms'], d['parity']['ok'])"
for i in 1 2 3; do
  run def_$i
  run gather_$i BLP_GROUP_GATHER=1
  run seg_$i BLP_SHORT_SEG=1
done
for i in 1 2; do
  BLP_CREATE_PROF=1 BLP_GRAPH_PROF=1 timeout -k 10 300 python bench.py --mode e2e --config c2 > gpurun_out/r05ab5_e2e_$i.json 2> gpurun_out/r05ab5_e2e_$i.err || { tail -20 gpurun_out/r05ab5_e2e_$i.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r05ab5_e2e_$i.json').read().strip().splitlines()[-1]);print('e2e', round(d['e2e_s'],4), {k: round(v,4) for k,v in d['phases_s'].items()}, d['graph_phase_detail_s'], d['ok'])"
done
