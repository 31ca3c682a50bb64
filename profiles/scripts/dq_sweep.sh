# config 2: business-side sources per dequeue (BLP_DQ) with wedge rows
set -o pipefail
cd $GRAFT_REPO_ROOT
for q in 1 2 3 4; do
  BLP_DQ=$q timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity > gpurun_out/dq_$q.json 2> gpurun_out/dq_$q.err || exit 1
done
