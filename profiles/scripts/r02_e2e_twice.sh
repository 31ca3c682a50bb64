#!/bin/bash
# similarity.main end to end at config 2, twice (file-phase variance), plus Yelp size
set -o pipefail
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" || exit 1
for r in 1 2; do
  timeout -k 10 600 python bench.py --mode e2e --config c2 > gpurun_out/r02_e2e_c2_$r.json 2> gpurun_out/r02_e2e_c2_$r.err || { tail -30 gpurun_out/r02_e2e_c2_$r.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['e2e_s'], d['phases_s'], d['ok'])" gpurun_out/r02_e2e_c2_$r.json
done
timeout -k 10 400 python bench.py --mode e2e --config yelp > gpurun_out/r02_e2e_yelp.json 2> gpurun_out/r02_e2e_yelp.err || { tail -30 gpurun_out/r02_e2e_yelp.err; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['e2e_s'], d['phases_s'], d['ok'])" gpurun_out/r02_e2e_yelp.json
