#!/bin/bash
# Round 6: config-5 phase clocks of k_score_split (libblp_prof.so, -DBLP_PROF; thread 0 of each
# workgroup): 0 claim, 1 build, 2 popcount + exact-distance removal, 3 short slices (the pair
# groups of a round, to the round's barrier), 4 the round's long slices. User pass alone.
# Build the library first: make -C bipartite-link-prediction_amd/csrc debug
#   DBG_OUT=../blp/libblp_prof.so DBG_FLAGS=-DBLP_PROF DBG_DIR=build_prof
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
BLP_LIB=$R/bipartite-link-prediction_amd/blp/libblp_prof.so BLP_PROF_READ=1 timeout -k 10 300 python -u bench.py --mode sharded --config c5 --sides user --steps 2 --warmup 1 --no-cpu-baseline --no-parity > gpurun_out/r06c5phase.json 2> gpurun_out/r06c5phase.err || { tail -20 gpurun_out/r06c5phase.err; exit 1; }
grep "prof" gpurun_out/r06c5phase.err
python -c "import json;d=json.loads(open('gpurun_out/r06c5phase.json').read().strip().splitlines()[-1]);print('user', round(d['ms_per_step'],2))"
