# config 2: wedge rows for the short-row (business) scorer; GPU tests, then the step with and
# without them and at two co-scheduling shares
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bw_on.json 2> gpurun_out/bw_on.err || exit 1
BLP_NO_WEDGE=1 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bw_off.json 2> gpurun_out/bw_off.err || exit 1
for c in 208 224; do
  BLP_COSCHED_CUS=$c timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bw_c$c.json 2> gpurun_out/bw_c$c.err || exit 1
done
timeout -k 10 300 python bench.py --no-cpu-baseline --sides business > gpurun_out/bw_bus.json 2> gpurun_out/bw_bus.err || exit 1
BLP_NO_WEDGE=1 timeout -k 10 300 python bench.py --no-cpu-baseline --sides business > gpurun_out/bw_bus_off.json 2> gpurun_out/bw_bus_off.err || exit 1
