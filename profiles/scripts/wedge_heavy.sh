# config 2: heavy business sources split into wedge-row slices; GPU tests, step on/off
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bh_on.json 2> gpurun_out/bh_on.err || exit 1
BLP_NO_WEDGE=1 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bh_off.json 2> gpurun_out/bh_off.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bh_on2.json 2> gpurun_out/bh_on2.err || exit 1
