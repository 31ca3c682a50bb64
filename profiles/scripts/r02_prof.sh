#!/bin/bash
# Round 2 profile of the default config-2 step: kernel trace + stats, FETCH_SIZE and WRITE_SIZE
# passes (summarize.py -> gpurun_out/$NAME.{json,md}), then counter passes that name the user
# scorer's binding unit (issue mix, LDS, waits, L2 hits) -> gpurun_out/${NAME}_pmc.txt.
# usage: bash profiles/scripts/r02_prof.sh NAME [bench args...]
set -o pipefail
R=$GRAFT_REPO_ROOT
NAME=$1
shift
ARGS="--steps 5 --warmup 1 --no-cpu-baseline --no-parity $*"
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
run() {  # pass-name, rocprofv3 args...
  local p=$1
  shift
  rm -rf $R/gpurun_out/prof_$p
  timeout -s KILL 240 rocprofv3 "$@" -d $R/gpurun_out/prof_$p -o $p -- python3 $R/bench.py $ARGS > $R/gpurun_out/${NAME}_$p.log 2>&1
}
run trace --kernel-trace --stats || exit 1
run fetch --pmc FETCH_SIZE || exit 1
run write --pmc WRITE_SIZE || exit 1
PROFILE_OUT=$R/gpurun_out python3 $R/profiles/summarize.py $NAME $(find $R/gpurun_out/prof_trace -name "*.db") $(find $R/gpurun_out/prof_fetch -name "*.db") $(find $R/gpurun_out/prof_write -name "*.db") > /dev/null || exit 1
run sq1 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE || exit 1
run sq2 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM || exit 1
run tcc --pmc TCC_HIT_sum TCC_MISS_sum || exit 1
python3 $R/profiles/pmc_report.py $(find $R/gpurun_out/prof_sq1 $R/gpurun_out/prof_sq2 $R/gpurun_out/prof_tcc -name "*.db") > $R/gpurun_out/${NAME}_pmc.txt 2>&1
head -60 $R/gpurun_out/${NAME}_pmc.txt
cat $R/gpurun_out/$NAME.md | head -30
