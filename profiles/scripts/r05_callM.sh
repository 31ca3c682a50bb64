#!/bin/bash
# Round 5 call M: is the remaining CSR-build stall (work queued on a stream that starts 20-30 ms
# late with the GPU idle, in about a third of the runs) streams sharing the process's hardware
# queues? Config-2 similarity.main with the image's 4 hardware queues per process (default)
# against 8 (GPU_MAX_HW_QUEUES=8), alternating, three each, slow HIP calls logged.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
e2e() {  # name, env...
  local n=$1
  shift
  env BLP_SLOW_HIP_MS=3 BLP_GRAPH_PROF=1 "$@" timeout -k 10 300 python bench.py --mode e2e --config c2 > gpurun_out/r05m_$n.json 2> gpurun_out/r05m_$n.err || { tail -20 gpurun_out/r05m_$n.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r05m_$n.json').read().strip().splitlines()[-1]);print('$n', round(d['e2e_s'],4), {k: round(v,4) for k,v in d['phases_s'].items()}, d['ok'])"
}
for i in 1 2 3; do
  e2e hwq4_$i
  e2e hwq8_$i GPU_MAX_HW_QUEUES=8
done
