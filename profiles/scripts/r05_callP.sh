#!/bin/bash
# Round 5 call P: the first batch of a pair on a highest-priority stream -- the similarity and
# headline tests; the config-2 bench line (default) against both batches from the normal pool
# (BLP_PAIR_SAME_PRIO=1), alternating, two each; a kernel trace of the default (the two passes'
# queue ids); config-2 similarity.main twice.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_similarity.py tests/test_gpu_headline.py > gpurun_out/r05p_tests.log 2>&1 || { tail -40 gpurun_out/r05p_tests.log; exit 1; }
tail -2 gpurun_out/r05p_tests.log
b() {  # name, env...
  local n=$1
  shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r05p_$n.json 2> gpurun_out/r05p_$n.err || { tail -20 gpurun_out/r05p_$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r05p_$n.json'));print('$n', round(d['ms_per_step'],3), d['kernels_ms'], d['parity']['ok'], d.get('including_batch_create'))"
}
for i in 1 2; do
  b hi_$i
  b same_$i BLP_PAIR_SAME_PRIO=1
done
for i in 1 2; do
  timeout -k 10 300 python bench.py --mode e2e --config c2 > gpurun_out/r05p_e2e_$i.json 2> gpurun_out/r05p_e2e_$i.err || { tail -20 gpurun_out/r05p_e2e_$i.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r05p_e2e_$i.json').read().strip().splitlines()[-1]);print('e2e', round(d['e2e_s'],4), {k: round(v,4) for k,v in d['phases_s'].items()}, d['ok'])"
done
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/prof_p
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_p -o p -- python3 $R/bench.py --no-cpu-baseline --no-parity --steps 3 --warmup 1 > $R/gpurun_out/r05p_trace.log 2>&1 || exit 1
mkdir -p $R/gpurun_out/r05p_trace
for f in $(find /tmp/prof_p -name "*kernel_trace.csv"); do gzip -c $f > $R/gpurun_out/r05p_trace/$(basename $f).gz; done
ls $R/gpurun_out/r05p_trace
