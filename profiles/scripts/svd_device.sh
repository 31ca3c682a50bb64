# config 4: device-resident top-k entry point; SVD tests, then the bench step on resident inputs
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest tests/test_gpu_svd.py -x -q --timeout 120 --timeout-method thread > gpurun_out/svd_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --mode svd > gpurun_out/svd_dev.json 2> gpurun_out/svd_dev.err || exit 1
