set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS -d $R/gpurun_out/pmc_tk1 -o sq -- python3 $R/bench.py --mode topk --topk-mask 1 --steps 1 --warmup 0 --no-cpu-baseline --no-parity > $R/gpurun_out/pmc_tk1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU -d $R/gpurun_out/pmc_tk2 -o f -- python3 $R/bench.py --mode topk --topk-mask 1 --steps 1 --warmup 0 --no-cpu-baseline --no-parity >> $R/gpurun_out/pmc_tk1.log 2>&1
python3 $R/profiles/pmc_report.py $(find $R/gpurun_out/pmc_tk1 $R/gpurun_out/pmc_tk2 -name "*.db") > $R/gpurun_out/pmc_tk_report.txt 2>&1
