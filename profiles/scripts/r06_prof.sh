#!/bin/bash
# Round 6 profile of one bench command (as r04_prof.sh): kernel trace + stats, FETCH_SIZE and
# WRITE_SIZE passes (summarize.py -> gpurun_out/$NAME.{json,md}), then SQ / TCC counter passes
# -> gpurun_out/${NAME}_pmc.txt. usage: bash profiles/scripts/r06_prof.sh NAME TIMEOUT [bench args...]
set -o pipefail
R=$GRAFT_REPO_ROOT
NAME=$1
TO=$2
shift 2
ARGS="--warmup 1 --no-cpu-baseline --no-parity $*"
mkdir -p $R/gpurun_out
P=/tmp/prof_$NAME
rm -rf $P
mkdir -p $P
cd /tmp && export TMPDIR=/tmp
run() {  # pass-name, rocprofv3 args...
  local p=$1
  shift
  timeout -s KILL $TO rocprofv3 "$@" -d $P/$p -o $p -- python3 $R/bench.py $ARGS > $R/gpurun_out/${NAME}_$p.log 2>&1
}
run trace --kernel-trace --stats || exit 1
run fetch --pmc FETCH_SIZE || exit 1
run write --pmc WRITE_SIZE || exit 1
PROFILE_OUT=$R/gpurun_out python3 $R/profiles/summarize.py $NAME $(find $P/trace -name "*.db") $(find $P/fetch -name "*.db") $(find $P/write -name "*.db") > /dev/null || exit 1
run sq1 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE || exit 1
run sq2 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM || exit 1
run tcc --pmc TCC_HIT_sum TCC_MISS_sum || exit 1
python3 $R/profiles/pmc_report.py $(find $P/sq1 $P/sq2 $P/tcc -name "*.db") > $R/gpurun_out/${NAME}_pmc.txt 2>&1
rm -rf $P
head -12 $R/gpurun_out/$NAME.md
