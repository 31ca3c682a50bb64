# config-4 top-k: number of column chunks (per-chunk top-k fills cost insertions: C k (1 + ln(N / (C k))))
set -o pipefail
cd $GRAFT_REPO_ROOT
for c in 3 4 6 13 14; do
  BLP_SVD_CHUNKS=$c timeout -k 10 200 python bench.py --mode svd --no-cpu-baseline --steps 10 > gpurun_out/svd_c$c.json 2> gpurun_out/svd_c$c.err || exit 1
done
