#!/bin/bash
# Round 5: large host buffers on transparent huge pages (default) against plain malloc / numpy
# (BLP_NO_THP=1) in config-2 similarity.main, and with the large copies explicitly registered
# (BLP_PIN_COPY=1), and with graph.txt uploaded from a file mapping (BLP_PARSE_MMAP=1, the
# round-4 path), alternating, two runs each; then the THP
# microbenchmark (first touch, fetch, unmap of 600 MB).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
e2e() {  # name, env...
  local n=$1
  shift
  env BLP_SLOW_HIP_MS=3 "$@" timeout -k 10 300 python bench.py --mode e2e --config c2 > gpurun_out/r05thp_$n.json 2> gpurun_out/r05thp_$n.err || { tail -20 gpurun_out/r05thp_$n.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r05thp_$n.json').read().strip().splitlines()[-1]);print('$n', round(d['e2e_s'],4), {k: round(v,4) for k,v in d['phases_s'].items()}, d['ok'])"
}
for i in 1 2; do
  e2e thp_$i
  e2e pin_$i BLP_PIN_COPY=1
  e2e mmap_$i BLP_PARSE_MMAP=1
  e2e nothp_$i BLP_NO_THP=1
done
timeout -k 10 120 python profiles/scripts/r05_hostmem2.py 600 > gpurun_out/r05_hostmem2.json || exit 1
cat gpurun_out/r05_hostmem2.json
