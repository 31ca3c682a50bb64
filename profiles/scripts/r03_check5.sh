#!/bin/bash
# Round 3, final check (after the hash/split partition of the active list): the whole GPU suite
# on the release build, smoke(), the default bench line, config 3, config 5 with parity, then
# rocprofv3 of the config-5 user pass (trace + FETCH/WRITE + SQ/TCC: r03_c5_v3, the summary
# bench.py's c5 line reads) and a kernel trace of the business pass (r03_c5_business_v3).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rs > gpurun_out/c5_gputest.log 2>&1 || { tail -40 gpurun_out/c5_gputest.log; exit 1; }
tail -3 gpurun_out/c5_gputest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/c5_smoke.log 2>&1 || { tail -20 gpurun_out/c5_smoke.log; exit 1; }
tail -1 gpurun_out/c5_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/c5_bench.json 2> gpurun_out/c5_bench.err || { tail -20 gpurun_out/c5_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/c5_bench.json'));print('bench', round(d['ms_per_step'],3), d['value'], d['kernels_ms'], d['parity']['u_cn_exact'], d['cpu_baseline'])"
timeout -k 10 300 python bench.py --mode topk --steps 5 --warmup 1 > gpurun_out/c5_topk.json 2> gpurun_out/c5_topk.err || { tail -20 gpurun_out/c5_topk.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/c5_topk.json'));print('topk', round(d['ms_per_step'],3), d['parity'])"
timeout -k 10 900 python -u bench.py --mode sharded --config c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c5_c5.json 2> gpurun_out/c5_c5.err || { tail -20 gpurun_out/c5_c5.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/c5_c5.json'));print('c5', round(d['ms_per_step'],3), d['roofline'].get('kernel_ms'), d.get('parity', {}).get('ok'))"
bash profiles/scripts/r03_prof.sh r03_c5_v3 --mode sharded --config c5 --sides user > gpurun_out/c5_prof_user.log 2>&1 || { tail -20 gpurun_out/c5_prof_user.log; exit 1; }
head -8 gpurun_out/r03_c5_v3.md | cut -c1-200
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/pb && timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d /tmp/pb -o trace -- python3 $R/bench.py --mode sharded --config c5 --steps 3 --warmup 1 --no-parity --no-cpu-baseline --sides business > $R/gpurun_out/c5_prof_bus.log 2>&1 || { tail -20 $R/gpurun_out/c5_prof_bus.log; exit 1; }
PROFILE_OUT=$R/gpurun_out python3 $R/profiles/summarize.py r03_c5_business_v3 $(find /tmp/pb -name "*.db") > /dev/null || exit 1
head -10 $R/gpurun_out/r03_c5_business_v3.md | cut -c1-200
