#!/bin/bash
# Round 5: LDS bank-conflict attribution of the config-2 user scorer. Three
# builds of the same kernel: libblp.so (full), libblp_exp1.so (-DBLP_EXP_PHASE=1: no pair scan),
# libblp_exp2.so (-DBLP_EXP_PHASE=2: no H2 build, so the scan reads an empty bitmap). One SQ pass
# each over the user side alone (bench.py --sides user) -> gpurun_out/r05_lds_attr_<v>_pmc.txt.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for v in full exp1 exp2; do
  P=/tmp/attr_$v
  rm -rf $P
  if [ $v = full ]; then LIB=$R/bipartite-link-prediction_amd/blp/libblp.so; else LIB=$R/bipartite-link-prediction_amd/blp/libblp_$v.so; fi
  BLP_LIB=$LIB timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_LDS -d $P -o attr -- python3 $R/bench.py --sides user --steps 5 --warmup 1 --no-cpu-baseline --no-parity --no-exchange > $R/gpurun_out/r05_lds_attr_$v.log 2>&1 || { tail -5 $R/gpurun_out/r05_lds_attr_$v.log; exit 1; }
  python3 $R/profiles/pmc_report.py $(find $P -name "*.db") > $R/gpurun_out/r05_lds_attr_${v}_pmc.txt 2>&1
  grep -A12 "k_score<1024" $R/gpurun_out/r05_lds_attr_${v}_pmc.txt | head -14
  rm -rf $P
done
