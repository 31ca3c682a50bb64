#!/bin/bash
# Round 4, check 7: the large scorer's packed-count variant (k_score PKO: 896-pair scan segments,
# no per-pair count array) -- the scorer tests (both variants via BLP_NO_PKO), the debug build,
# then an alternating A/B of the config-2 step (PKO vs BLP_NO_PKO=1) and the default bench line.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_similarity.py tests/test_gpu_headline.py tests/test_gpu_debug.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04c7_gputest.log 2>&1 || { tail -60 gpurun_out/r04c7_gputest.log; exit 1; }
tail -1 gpurun_out/r04c7_gputest.log
ab() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --no-exchange --steps 20 --warmup 3 > gpurun_out/ab7_$name.json 2> gpurun_out/ab7_$name.err || { tail -5 gpurun_out/ab7_$name.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab7_$name.json'));print('$name', round(d['ms_per_step'],4), {k: round(v['score_ms'],3) for k,v in d['kernels_ms'].items()}, d.get('parity',{}).get('ok'))"
}
ab pko1 BLP_X=0 && ab gen1 BLP_NO_PKO=1 && ab pko2 BLP_X=0 && ab gen2 BLP_NO_PKO=1 && ab pko3 BLP_X=0 && ab gen3 BLP_NO_PKO=1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/r04c7_bench.json 2> gpurun_out/r04c7_bench.err || { tail -20 gpurun_out/r04c7_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r04c7_bench.json'));print('bench', round(d['ms_per_step'],3), d['value'], d['kernels_ms'], d['parity']['ok'], d['roofline']['kernel'])"
bash profiles/scripts/r04_prof.sh r04_v7_bench || { echo "c2 profile failed"; exit 1; }
head -8 gpurun_out/r04_v7_bench.md
grep -A18 "31744" gpurun_out/r04_v7_bench_pmc.txt | head -20
