#!/bin/bash
# Round 3: similarity.main end to end (config 2, config 1 shape), with the native edge loader,
# the overlapped examples parse and the concurrent score files (A/B: one writer); user side on
# the chunk-parallel scorer; item grouping with staged records vs buckets; (two 64 KiB chunks, two workgroups per CU) vs the large scorer.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
e() {  # name, env..., -- args
  local n=$1; shift
  timeout -k 10 600 python -u bench.py --mode e2e "$@" > gpurun_out/e11_$n.json 2> gpurun_out/e11_$n.err || { tail -20 gpurun_out/e11_$n.err; return 1; }
  tail -1 gpurun_out/e11_$n.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$n', round(d['e2e_s'],3), d['phases_s'], d.get('graph_phase_detail_s'), d['ok'])"
}
BLP_INGEST_PROF=1 e c2 --config c2 || exit 1
grep blp_edges_load gpurun_out/e11_c2.err
BLP_FILE_WRITERS=1 e c2_w1 --config c2 || exit 1
e c2_b --config c2 || exit 1
e yelp --config yelp || exit 1
q() {  # name, args...
  local n=$1; shift
  timeout -k 10 600 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/e11_$n.json 2> gpurun_out/e11_$n.err || { tail -20 gpurun_out/e11_$n.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/e11_$n.json'));print('$n', round(d['ms_per_step'],3), d.get('kernels_ms'))"
}
q c2bench --steps 20 --warmup 3 || exit 1
BLP_GROUP_BUCKETS=1 q c2_buckets --steps 20 --warmup 3 --no-parity || exit 1
q c2_user --steps 20 --warmup 3 --no-parity --sides user || exit 1
BLP_SPLIT=2 BLP_SPLIT_BIG=0 q c2_user_split2 --steps 20 --warmup 3 --no-parity --sides user || exit 1
BLP_SPLIT=2 BLP_SPLIT_BIG=0 BLP_SPLIT_SHORT=0 q c2_user_split2ns --steps 20 --warmup 3 --no-parity --sides user || exit 1
