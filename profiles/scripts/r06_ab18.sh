#!/bin/bash
# Round 6, A/B 18, alternating on one box: config 2, the user scorer's first pair segment
# prefetched in two stages (y with the source header, rp[y] once the dense-row OR is issued, so
# the second hop hides behind the sparse build; libblp.so) against one stage (both hops at the
# header: the wave waits for y before the build; libblp_prev.so = HEAD); the next segment's
# prefetch split the same way (y before the offsets' barriers, rp[y] after). First the similarity,
# headline and debug tests; the first new arm checks parity.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
L=$R/bipartite-link-prediction_amd/blp
timeout -k 10 300 python -u -m pytest tests/test_gpu_similarity.py tests/test_gpu_headline.py tests/test_gpu_debug.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06ab18_tests.log 2>&1 || { tail -30 gpurun_out/r06ab18_tests.log; exit 1; }
tail -1 gpurun_out/r06ab18_tests.log
run() {  # name lib [extra]
  BLP_LIB=$L/$2 timeout -k 10 300 python bench.py --no-cpu-baseline --no-exchange ${3:---no-parity} > gpurun_out/r06ab18_$1.json 2> gpurun_out/r06ab18_$1.err || { tail -20 gpurun_out/r06ab18_$1.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r06ab18_$1.json'));print('$1', round(d['ms_per_step'],4), (d.get('parity') or {}).get('ok'), {k: {kk: round(vv, 4) for kk, vv in x.items()} for k, x in d['kernels_ms'].items()})"
}
run new_0 libblp.so --steps=20 || exit 1
for round in 1 2 3 4; do
  run new_$round libblp.so && run prev_$round libblp_prev.so || exit 1
done
