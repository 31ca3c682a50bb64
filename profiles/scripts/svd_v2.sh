# config-4 top-k after the bitonic compaction: tests, then default chunks vs overrides
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest tests/test_gpu_svd.py -x -q --timeout 120 --timeout-method thread > gpurun_out/svd_tests.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --mode svd --no-cpu-baseline --steps 10 > gpurun_out/svd_d.json 2> gpurun_out/svd_d.err || exit 1
for c in 2 4 6 13; do
  BLP_SVD_CHUNKS=$c timeout -k 10 200 python bench.py --mode svd --no-cpu-baseline --steps 10 > gpurun_out/svd_c$c.json 2> gpurun_out/svd_c$c.err || exit 1
done
