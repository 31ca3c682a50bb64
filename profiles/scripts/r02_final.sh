#!/bin/bash
# Round 2 end-to-end evidence run: GPU suite, smoke, the default bench (config 2), config 3, 4,
# end-to-end configs 1 and 2 -> gpurun_out/r02f_*.json. Each step has its own time limit; the
# first failure ends the script.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
export TMPDIR=${TMPDIR:-/tmp}
step() {  # name, seconds, command...
  local n=$1 t=$2
  shift 2
  timeout -k 10 $t "$@" > gpurun_out/r02f_$n.json 2> gpurun_out/r02f_$n.err || { echo "FAILED $n"; tail -20 gpurun_out/r02f_$n.err; exit 1; }
  echo "== $n"; tail -c 2500 gpurun_out/r02f_$n.json
}
step tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
step bench 300 python bench.py
step topk 400 python bench.py --mode topk
step svd 600 python bench.py --mode svd
step e2e_yelp 300 python bench.py --mode e2e --config yelp
step e2e_c2 400 python bench.py --mode e2e --config c2
