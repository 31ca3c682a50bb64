set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python bench.py > gpurun_out/bench_v16.json 2> gpurun_out/bench_v16.err || exit 1
timeout -k 10 200 python bench.py --mode svd --no-cpu-baseline --steps 10 > gpurun_out/svd_rt2.json 2> gpurun_out/svd_rt2.err || exit 1
BLP_SVD_RT=1 timeout -k 10 200 python bench.py --mode svd --no-cpu-baseline --steps 10 > gpurun_out/svd_rt1.json 2> gpurun_out/svd_rt1.err || exit 1
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/svdf2 $R/gpurun_out/svdf1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/svdf2 -o f -- python3 $R/bench.py --mode svd --no-cpu-baseline --no-parity --steps 3 --warmup 1 > $R/gpurun_out/svdf2.log 2>&1 || exit 1
BLP_SVD_RT=1 timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/svdf1 -o f -- python3 $R/bench.py --mode svd --no-cpu-baseline --no-parity --steps 3 --warmup 1 > $R/gpurun_out/svdf1.log 2>&1 || exit 1
