#!/bin/bash
# Round 5 profiles at HEAD (1/2): config 2's bench command (r05_v1_bench: the line's roofline
# provenance) and config 5's user pass alone (r05_c5_user: --sides user).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
bash profiles/scripts/r05_prof.sh r05_v1_bench 300 --steps 5 || exit 1
bash profiles/scripts/r05_prof.sh r05_c5_user 300 --mode sharded --config c5 --steps 2 --sides user || exit 1
