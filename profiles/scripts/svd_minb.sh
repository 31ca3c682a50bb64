# config-4 top-k at 3 blocks (12 waves) per CU: tests, default chunks (fills 768 slots once), overrides
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest tests/test_gpu_svd.py -x -q --timeout 120 --timeout-method thread > gpurun_out/svd_tests.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --mode svd --no-cpu-baseline --steps 10 > gpurun_out/svd_m.json 2> gpurun_out/svd_m.err || exit 1
for c in 3 5; do
  BLP_SVD_CHUNKS=$c timeout -k 10 200 python bench.py --mode svd --no-cpu-baseline --steps 10 > gpurun_out/svd_m$c.json 2> gpurun_out/svd_m$c.err || exit 1
done
