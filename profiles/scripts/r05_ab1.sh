#!/bin/bash
# Round 5 A/B 1: business grouping with y only (k_item_write_ids; default) against the 16-byte
# row-bound records (BLP_GROUP_ROWS=1), alternating on one box. One full-parity bench first.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r05ab1_parity.json 2> gpurun_out/r05ab1_parity.err || { tail -20 gpurun_out/r05ab1_parity.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r05ab1_parity.json'));print('parity bench', round(d['ms_per_step'],3), d['kernels_ms'], d['parity']['ok'])"
for i in 1 2 3; do
  for v in new old; do
    if [ $v = old ]; then export BLP_GROUP_ROWS=1; else unset BLP_GROUP_ROWS; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity --steps 30 > gpurun_out/r05ab1_${v}_$i.json 2> gpurun_out/r05ab1_${v}_$i.err || { tail -20 gpurun_out/r05ab1_${v}_$i.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/r05ab1_${v}_$i.json'));print('$v', $i, round(d['ms_per_step'],3), {k:{a:round(b,3) for a,b in v.items()} for k,v in d['kernels_ms'].items()})"
  done
done
