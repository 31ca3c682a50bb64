#!/bin/bash
# Round 5 call E: the whole GPU suite at HEAD (per-wave top-k selection by default, huge-page host
# buffers, threaded graph.txt read, two-pass score files, registered-copy helper); then config-2
# similarity.main with the stream prewarm topping the pool up and activating new streams
# (default) against always creating four (BLP_PREWARM_ALWAYS=1), alternating, three each.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r05e_gputest.log 2>&1 || { tail -40 gpurun_out/r05e_gputest.log; exit 1; }
tail -3 gpurun_out/r05e_gputest.log
e2e() {  # name, env...
  local n=$1
  shift
  env BLP_SLOW_HIP_MS=3 "$@" timeout -k 10 300 python bench.py --mode e2e --config c2 > gpurun_out/r05pw_$n.json 2> gpurun_out/r05pw_$n.err || { tail -20 gpurun_out/r05pw_$n.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r05pw_$n.json').read().strip().splitlines()[-1]);print('$n', round(d['e2e_s'],4), {k: round(v,4) for k,v in d['phases_s'].items()}, d['ok'])"
}
for i in 1 2 3; do
  e2e top_$i
  e2e always_$i BLP_PREWARM_ALWAYS=1
done
