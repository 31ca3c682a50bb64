# config 2: bucket-group counting pass unrolled; GPU tests, then the step twice
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bg_1.json 2> gpurun_out/bg_1.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bg_2.json 2> gpurun_out/bg_2.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --sides business > gpurun_out/bg_bus.json 2> gpurun_out/bg_bus.err || exit 1
