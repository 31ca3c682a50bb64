# config 2: user-scorer CU share sweep (BLP_COSCHED_CUS) after the wedge rows
set -o pipefail
cd $GRAFT_REPO_ROOT
for c in 168 180 192 204 216; do
  BLP_COSCHED_CUS=$c timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity > gpurun_out/cs_$c.json 2> gpurun_out/cs_$c.err || exit 1
done
