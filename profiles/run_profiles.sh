# Profile one bench command: rocprofv3 kernel trace + stats, then separate FETCH_SIZE and
# WRITE_SIZE passes (they cannot share a pass on gfx950), summarised by summarize.py into
# gpurun_out/<NAME>.{json,md} (copy into profiles/ to commit).
# usage (on the GPU box): bash profiles/run_profiles.sh NAME [bench.py args...]
set -e
R=$GRAFT_REPO_ROOT
NAME=$1
shift
cd /tmp && export TMPDIR=/tmp
for pass in trace fetch write; do rm -rf $R/gpurun_out/prof_$pass; done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_trace -o trace -- python3 $R/bench.py "$@" > $R/gpurun_out/${NAME}_trace.log 2>&1
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/prof_fetch -o fetch -- python3 $R/bench.py "$@" > $R/gpurun_out/${NAME}_fetch.log 2>&1
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/prof_write -o write -- python3 $R/bench.py "$@" > $R/gpurun_out/${NAME}_write.log 2>&1
PROFILE_OUT=$R/gpurun_out python3 $R/profiles/summarize.py $NAME $(find $R/gpurun_out/prof_trace -name "*.db") $(find $R/gpurun_out/prof_fetch -name "*.db") $(find $R/gpurun_out/prof_write -name "*.db") > /dev/null
