#!/bin/bash
# Round 6, check 3: the business pass on the dense wedge-set index (k_score_wset). The wedge-set
# and headline tests first, then the config-2 step: the default (wedge-set batches serialised
# after the user pass, which takes the whole chip) against the concurrent variant at several user
# CU shares and the grouped path (BLP_NO_WSET=1); full parity on the default; then the GPU suite.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_similarity.py -k "wedge_set_path or kernel_paths" tests/test_gpu_headline.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r06c3_first.log 2>&1 || { tail -40 gpurun_out/r06c3_first.log; exit 1; }
tail -2 gpurun_out/r06c3_first.log
timeout -k 10 300 python bench.py --no-exchange > gpurun_out/r06c3_bench.json 2> gpurun_out/r06c3_bench.err || { tail -20 gpurun_out/r06c3_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r06c3_bench.json'));print('bench', round(d['ms_per_step'],4), d['value'], d['kernels_ms'], d['parity']['ok'])"
for round in 1 2; do
  for v in serial par:256 par:240 par:224 par:208 par:192 nowset:0; do
    name=${v%%:*}; cus=${v##*:}
    env="BLP_WSET_SERIAL=1"
    [ $name = par ] && env="BLP_WSET_SERIAL=0 BLP_COSCHED_CUS=$cus"
    [ $name = nowset ] && env="BLP_NO_WSET=1"
    env $env timeout -k 10 300 python bench.py --no-cpu-baseline --no-exchange --no-parity > gpurun_out/r06c3_${name}_${cus}_$round.json 2> gpurun_out/r06c3_${name}_${cus}_$round.err || { tail -20 gpurun_out/r06c3_${name}_${cus}_$round.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r06c3_${name}_${cus}_$round.json'));print('$name', '$cus', $round, round(d['ms_per_step'],4), {k: {kk: round(vv, 4) for kk, vv in x.items()} for k, x in d['kernels_ms'].items()})"
  done
done
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rs > gpurun_out/r06c3_gputest.log 2>&1 || { tail -40 gpurun_out/r06c3_gputest.log; exit 1; }
tail -3 gpurun_out/r06c3_gputest.log
