#!/bin/bash
# Round 4, check 5: config 4 re-profiled after the dense top-k's chunk cap (the 64-user host
# call's merge), its bench line; config-2 A/B of this round's scorer changes against the
# round-3 order (libblp_exp_old.so: -DBLP_EXP_NOCLEAN -DBLP_EXP_ESC), alternating on one box;
# experiment 1 (user side: LARGE block scorer vs two half-universe chunks); experiment 2
# (config-5 user pass, chunk partials' atomics in L2 vs device scope).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_similarity.py tests/test_gpu_headline.py tests/test_gpu_svd.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04c5_gputest.log 2>&1 || { tail -40 gpurun_out/r04c5_gputest.log; exit 1; }
tail -1 gpurun_out/r04c5_gputest.log
BLP_GRAPH_PROF=1 timeout -k 10 300 python bench.py --mode e2e --config c2 > gpurun_out/r04c5_e2e.json 2> gpurun_out/r04c5_e2e.err || { tail -20 gpurun_out/r04c5_e2e.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r04c5_e2e.json').read().strip().splitlines()[-1]);print('e2e', d['e2e_s'], d['phases_s'], d['graph_phase_detail_s'], d['ok'])"
grep -E "graph_finish" gpurun_out/r04c5_e2e.err | tail -8
bash profiles/scripts/r04_prof.sh r04_svd_c4 --mode svd || { echo "svd profile failed"; exit 1; }
head -8 gpurun_out/r04_svd_c4.md
timeout -k 10 300 python bench.py --mode svd > gpurun_out/r04c5_svd.json 2> gpurun_out/r04c5_svd.err || { tail -20 gpurun_out/r04c5_svd.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r04c5_svd.json'));print('svd', round(d['ms_per_step'],3), d['value'], d['roofline'], d['cpu_baseline'], d['parity'])"
ab() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --no-exchange --steps 20 --warmup 3 > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err || { tail -5 gpurun_out/ab_$name.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab_$name.json'));print('$name', round(d['ms_per_step'],4), {k: round(v['score_ms'],3) for k,v in d['kernels_ms'].items()}, d.get('parity',{}).get('ok'))"
}
OLD=$R/bipartite-link-prediction_amd/blp/libblp_exp_old.so
ab new1 BLP_X=0 && ab old1 BLP_LIB=$OLD && ab new2 BLP_X=0 && ab old2 BLP_LIB=$OLD && ab new3 BLP_X=0 && ab old3 BLP_LIB=$OLD || exit 1
bash profiles/scripts/r04_exp1.sh || exit 1
bash profiles/scripts/r04_exp2.sh
