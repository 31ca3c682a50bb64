# config-4 top-k: register-threshold epilogue; tests first, then the bench variants
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest tests/test_gpu_svd.py -x -q --timeout 120 --timeout-method thread > gpurun_out/svd_tests.log 2>&1 || exit 1
BLP_SVD_RT=2 timeout -k 10 200 python -u -m pytest tests/test_gpu_svd.py -x -q --timeout 120 --timeout-method thread > gpurun_out/svd_tests_rt2.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --mode svd --no-cpu-baseline --steps 10 > gpurun_out/svd_e1.json 2> gpurun_out/svd_e1.err || exit 1
BLP_SVD_RT=2 timeout -k 10 200 python bench.py --mode svd --no-cpu-baseline --steps 10 > gpurun_out/svd_e2.json 2> gpurun_out/svd_e2.err || exit 1
BLP_SVD_KC=2 timeout -k 10 200 python bench.py --mode svd --no-cpu-baseline --steps 10 > gpurun_out/svd_e3.json 2> gpurun_out/svd_e3.err || exit 1
