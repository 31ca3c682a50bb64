# config 2: short-row scorer with the first segment's pair metadata loaded before the build
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_similarity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sim_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bp_1.json 2> gpurun_out/bp_1.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --sides business > gpurun_out/bp_bus.json 2> gpurun_out/bp_bus.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bp_2.json 2> gpurun_out/bp_2.err || exit 1
