#!/bin/bash
# Round 5 call L: blp_batch_create_pair planning both batches concurrently (one upload into shared
# device arrays) -- the pair tests (concurrent and serial), the similarity suite; then config-2
# similarity.main with the create-stage timers, concurrent (default) against serial
# (BLP_PAIR_SERIAL=1), alternating, three each; then the default bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_similarity.py tests/test_gpu_headline.py > gpurun_out/r05l_tests.log 2>&1 || { tail -40 gpurun_out/r05l_tests.log; exit 1; }
tail -2 gpurun_out/r05l_tests.log
e2e() {  # name, env...
  local n=$1
  shift
  env BLP_SLOW_HIP_MS=3 BLP_CREATE_PROF=1 "$@" timeout -k 10 300 python bench.py --mode e2e --config c2 > gpurun_out/r05l_$n.json 2> gpurun_out/r05l_$n.err || { tail -20 gpurun_out/r05l_$n.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r05l_$n.json').read().strip().splitlines()[-1]);print('$n', round(d['e2e_s'],4), {k: round(v,4) for k,v in d['phases_s'].items()}, d['ok'])"
}
for i in 1 2 3; do
  e2e conc_$i
  e2e serial_$i BLP_PAIR_SERIAL=1
done
timeout -k 10 300 python bench.py > gpurun_out/r05l_bench.json 2> gpurun_out/r05l_bench.err || { tail -20 gpurun_out/r05l_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r05l_bench.json'));print('bench', round(d['ms_per_step'],3), d['value'], d['parity']['ok'], d.get('including_batch_create'))"
