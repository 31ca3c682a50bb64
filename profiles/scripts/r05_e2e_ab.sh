#!/bin/bash
# Round 5: config 2 end to end, the stream prewarm (default) against the HIP runtime start only
# (BLP_NO_PREWARM=1), alternating on one box, three runs each; stage timers on stderr.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
e2e() {  # name, env...
  local n=$1
  shift
  env BLP_CREATE_PROF=1 BLP_GRAPH_PROF=1 "$@" timeout -k 10 300 python bench.py --mode e2e --config c2 > gpurun_out/r05e2e_$n.json 2> gpurun_out/r05e2e_$n.err || { tail -20 gpurun_out/r05e2e_$n.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r05e2e_$n.json').read().strip().splitlines()[-1]);print('$n', round(d['e2e_s'],4), {k: round(v,4) for k,v in d['phases_s'].items()}, {k: round(v,4) for k,v in d['graph_phase_detail_s'].items()}, d['ok'])"
}
for i in 1 2 3; do
  e2e pre_$i
  e2e nopre_$i BLP_NO_PREWARM=1
done
grep -E "blp_batch_create|graph_finish" gpurun_out/r05e2e_pre_3.err | head -30
