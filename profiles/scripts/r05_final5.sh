#!/bin/bash
# Round 5, final check 5 at HEAD (after the last code change): the whole GPU suite, smoke(), the
# default bench line (its kernels are those profiled in r05_v2_bench), config-2 similarity.main
# three times and config 1 once.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rs > gpurun_out/r05fin5_gputest.log 2>&1 || { tail -60 gpurun_out/r05fin5_gputest.log; exit 1; }
tail -3 gpurun_out/r05fin5_gputest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05fin5_smoke.log 2>&1 || { tail -20 gpurun_out/r05fin5_smoke.log; exit 1; }
tail -1 gpurun_out/r05fin5_smoke.log


timeout -k 10 300 python bench.py > gpurun_out/r05fin5_bench.json 2> gpurun_out/r05fin5_bench.err || { tail -20 gpurun_out/r05fin5_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r05fin5_bench.json'));print('bench', round(d['ms_per_step'],3), d['value'], d['kernels_ms'], d['parity']['ok'], d['roofline'], d.get('including_batch_create'))"
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --mode e2e --config c2 > gpurun_out/r05fin5_e2e_$i.json 2> gpurun_out/r05fin5_e2e_$i.err || { tail -20 gpurun_out/r05fin5_e2e_$i.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r05fin5_e2e_$i.json').read().strip().splitlines()[-1]);print('e2e', round(d['e2e_s'],4), {k: round(v,4) for k,v in d['phases_s'].items()}, d['ok'])"
done
BLP_CREATE_PROF=1 timeout -k 10 300 python bench.py --mode e2e --config c2 > gpurun_out/r05fin5_e2e_cprof.json 2> gpurun_out/r05fin5_e2e_cprof.err || { tail -20 gpurun_out/r05fin5_e2e_cprof.err; exit 1; }
grep -i "create\|upload\|plan\|sources\|heavy\|wbm\|split\|buffers\|pairs" gpurun_out/r05fin5_e2e_cprof.err | head -30
timeout -k 10 600 python bench.py --mode topk > gpurun_out/r05fin5_topk.json 2> gpurun_out/r05fin5_topk.err || { tail -20 gpurun_out/r05fin5_topk.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r05fin5_topk.json').read().strip().splitlines()[-1]);print('c3', round(d['ms_per_step'],3), d['value'], d.get('parity'), d['roofline'])"
timeout -k 10 300 python bench.py --mode e2e --config yelp > gpurun_out/r05fin5_e2e_yelp.json 2> gpurun_out/r05fin5_e2e_yelp.err || { tail -20 gpurun_out/r05fin5_e2e_yelp.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r05fin5_e2e_yelp.json').read().strip().splitlines()[-1]);print('e2e yelp', round(d['e2e_s'],4), d['ok'])"
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/prof_f5
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_f5 -o f5 -- python3 $R/bench.py --no-cpu-baseline --no-parity > $R/gpurun_out/r05fin5_prof.log 2>&1 || exit 1
mkdir -p $R/gpurun_out/r05fin5_prof
for f in $(find /tmp/prof_f5 -name "*stats.csv"); do cp $f $R/gpurun_out/r05fin5_prof/; done
ls $R/gpurun_out/r05fin5_prof
