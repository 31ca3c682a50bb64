#!/bin/bash
# Round 4, check 6: the whole GPU suite at HEAD, the default bench line, config 2 end to end
# with 3 and 6 concurrent score-file writers, and the config-2 profile (trace + FETCH/WRITE +
# SQ/TCC passes) the bench line's roofline cites.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rs > gpurun_out/r04c6_gputest.log 2>&1 || { tail -60 gpurun_out/r04c6_gputest.log; exit 1; }
tail -3 gpurun_out/r04c6_gputest.log
timeout -k 10 300 python bench.py > gpurun_out/r04c6_bench.json 2> gpurun_out/r04c6_bench.err || { tail -20 gpurun_out/r04c6_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r04c6_bench.json'));print('bench', round(d['ms_per_step'],3), d['value'], d['kernels_ms'], d['parity']['ok'], d['roofline'])"
for w in 3 6 3 6; do
  BLP_FILE_WRITERS=$w timeout -k 10 300 python bench.py --mode e2e --config c2 > gpurun_out/r04c6_e2e_w$w.json 2> gpurun_out/r04c6_e2e_w$w.err || { tail -20 gpurun_out/r04c6_e2e_w$w.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r04c6_e2e_w$w.json').read().strip().splitlines()[-1]);print('e2e writers=$w', round(d['e2e_s'],4), {k: round(v,4) for k,v in d['phases_s'].items()}, d['ok'])"
done
bash profiles/scripts/r04_prof.sh r04_c2 || { echo "c2 profile failed"; exit 1; }
head -10 gpurun_out/r04_c2.md
bash profiles/scripts/r04_exp3.sh
