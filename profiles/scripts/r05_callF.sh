#!/bin/bash
# Round 5 call F: the whole GPU suite with the device scratch cache; config-2 similarity.main with
# the cache (default) against without it (BLP_DEV_CACHE_MB=0), alternating, three each, slow HIP
# calls logged; then the default bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r05f_gputest.log 2>&1 || { tail -40 gpurun_out/r05f_gputest.log; exit 1; }
tail -3 gpurun_out/r05f_gputest.log
e2e() {  # name, env...
  local n=$1
  shift
  env BLP_SLOW_HIP_MS=3 "$@" timeout -k 10 300 python bench.py --mode e2e --config c2 > gpurun_out/r05dc_$n.json 2> gpurun_out/r05dc_$n.err || { tail -20 gpurun_out/r05dc_$n.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r05dc_$n.json').read().strip().splitlines()[-1]);print('$n', round(d['e2e_s'],4), {k: round(v,4) for k,v in d['phases_s'].items()}, d['ok'])"
}
for i in 1 2 3; do
  e2e cache_$i
  e2e nocache_$i BLP_DEV_CACHE_MB=0
done
timeout -k 10 300 python bench.py > gpurun_out/r05f_bench.json 2> gpurun_out/r05f_bench.err || { tail -20 gpurun_out/r05f_bench.err; exit 1; }
tail -1 gpurun_out/r05f_bench.json | cut -c1-600
