#!/bin/bash
# Round 5 profiles at HEAD (2/2): config 5's business pass alone (r05_c5_business) and config 3's
# top-k step (r05_topk_v1).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
bash profiles/scripts/r05_prof.sh r05_c5_business 300 --mode sharded --config c5 --steps 2 --sides business || exit 1
bash profiles/scripts/r05_prof.sh r05_topk_v1 300 --mode topk --steps 5 || exit 1
