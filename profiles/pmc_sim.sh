# PMC passes over the config-2 similarity bench (SQ issue/wait mix, LDS, L2-miss bytes).
set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS -d $R/gpurun_out/pmc_sim1 -o sq -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity > $R/gpurun_out/pmc_sim.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU -d $R/gpurun_out/pmc_sim2 -o f -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity >> $R/gpurun_out/pmc_sim.log 2>&1
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCP_TCC_READ_REQ_sum -d $R/gpurun_out/pmc_sim3 -o c -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-parity >> $R/gpurun_out/pmc_sim.log 2>&1 || true
python3 $R/profiles/pmc_report.py $(find $R/gpurun_out/pmc_sim1 $R/gpurun_out/pmc_sim2 $R/gpurun_out/pmc_sim3 -name "*.db") > $R/gpurun_out/pmc_sim_report.txt 2>&1
