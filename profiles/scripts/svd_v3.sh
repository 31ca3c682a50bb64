# config-4 top-k: branch-free epilogue; tests (both tilings), default and RT=2 timings
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest tests/test_gpu_svd.py -x -q --timeout 120 --timeout-method thread > gpurun_out/svd_tests.log 2>&1 || exit 1
BLP_SVD_RT=2 timeout -k 10 200 python -u -m pytest tests/test_gpu_svd.py -x -q --timeout 120 --timeout-method thread > gpurun_out/svd_tests_rt2.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --mode svd --no-cpu-baseline --steps 10 > gpurun_out/svd_d.json 2> gpurun_out/svd_d.err || exit 1
BLP_SVD_RT=2 timeout -k 10 200 python bench.py --mode svd --no-cpu-baseline --steps 10 > gpurun_out/svd_rt2.json 2> gpurun_out/svd_rt2.err || exit 1
BLP_SVD_EXP=1 timeout -k 10 200 python bench.py --mode svd --no-cpu-baseline --no-parity --steps 10 > gpurun_out/svd_exp1.json 2> gpurun_out/svd_exp1.err || exit 1
