# config-4 top-k: epilogue-free timing experiment + one SQ counter pass over the real kernel
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
BLP_SVD_EXP=1 timeout -k 10 200 python bench.py --mode svd --no-cpu-baseline --no-parity --steps 10 > gpurun_out/svd_exp1.json 2> gpurun_out/svd_exp1.err || exit 1
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/svdsq
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_VALU_MFMA_BUSY_CYCLES -d $R/gpurun_out/svdsq -o f -- python3 $R/bench.py --mode svd --no-cpu-baseline --no-parity --steps 2 --warmup 1 > $R/gpurun_out/svdsq.log 2>&1 || exit 1
