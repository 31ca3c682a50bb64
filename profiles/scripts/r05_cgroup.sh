#!/bin/bash
# Round 5: is the e2e run's host stall CPU-quota throttling? The box's cgroup CPU limit and its
# throttling counters before and after one config-2 similarity.main run.
set -o pipefail
cd $GRAFT_REPO_ROOT || exit 1
mkdir -p gpurun_out
{
  echo "nproc $(nproc) affinity $(python -c 'import os;print(len(os.sched_getaffinity(0)))')"
  for f in /sys/fs/cgroup/cpu.max /sys/fs/cgroup/cpu.max.burst /sys/fs/cgroup/cpu/cpu.cfs_quota_us /sys/fs/cgroup/cpu/cpu.cfs_period_us; do
    [ -r $f ] && echo "$f: $(cat $f)"
  done
  cat /proc/self/cgroup
  echo "--- cpu.stat before"
  cat /sys/fs/cgroup/cpu.stat 2>/dev/null || cat /sys/fs/cgroup/cpu/cpu.stat 2>/dev/null
} > gpurun_out/r05_cgroup.txt 2>&1
for i in 1 2; do
  BLP_GRAPH_PROF=1 timeout -k 10 300 python bench.py --mode e2e --config c2 > gpurun_out/r05_cgroup_e2e_$i.json 2> gpurun_out/r05_cgroup_e2e_$i.err || exit 1
  { echo "--- cpu.stat after run $i"; cat /sys/fs/cgroup/cpu.stat 2>/dev/null || cat /sys/fs/cgroup/cpu/cpu.stat 2>/dev/null; } >> gpurun_out/r05_cgroup.txt
done
cat gpurun_out/r05_cgroup.txt
