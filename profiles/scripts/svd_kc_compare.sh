# config-4 top-k variants + the fp64 MFMA rate microbenchmark (run on the GPU box)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 60 profiles/scripts/mfma_f64_peak > gpurun_out/mfma_f64_peak.txt 2>&1 || exit 1
timeout -k 10 200 python -u -m pytest tests/test_gpu_svd.py -x -q --timeout 120 --timeout-method thread > gpurun_out/svd_tests.log 2>&1 || exit 1
BLP_SVD_KC=2 timeout -k 10 200 python -u -m pytest tests/test_gpu_svd.py -x -q --timeout 120 --timeout-method thread > gpurun_out/svd_tests_kc2.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --mode svd --no-cpu-baseline --steps 10 > gpurun_out/svd_kc1.json 2> gpurun_out/svd_kc1.err || exit 1
BLP_SVD_KC=2 timeout -k 10 200 python bench.py --mode svd --no-cpu-baseline --steps 10 > gpurun_out/svd_kc2.json 2> gpurun_out/svd_kc2.err || exit 1
