#!/bin/bash
# Round 5 call AE2: the same counters after the scatter lost its key array (the
# round-6 lead): FETCH_SIZE, WRITE_SIZE (TCC) and an SQ pass, each its own run of the
# default bench (--steps 5, no parity, no CPU baseline).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/pmc_ae2_1 /tmp/pmc_ae2_2 /tmp/pmc_ae2_3
# FETCH_SIZE takes 3 of the 4 TCC counters and WRITE_SIZE 2: one pass each
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d /tmp/pmc_ae2_1 -o f -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-parity > $R/gpurun_out/r05ae2_f.log 2>&1 || { tail -5 $R/gpurun_out/r05ae2_f.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d /tmp/pmc_ae2_3 -o w -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-parity > $R/gpurun_out/r05ae2_w.log 2>&1 || { tail -5 $R/gpurun_out/r05ae2_w.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_VMEM_RD -d /tmp/pmc_ae2_2 -o sq -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-parity > $R/gpurun_out/r05ae2_sq.log 2>&1 || { tail -5 $R/gpurun_out/r05ae2_sq.log; exit 1; }
python3 $R/profiles/pmc_report.py $(find /tmp/pmc_ae2_1 /tmp/pmc_ae2_2 /tmp/pmc_ae2_3 -name "*.db") > $R/gpurun_out/r05ae2_pmc.txt 2>&1
head -80 $R/gpurun_out/r05ae2_pmc.txt
