#!/bin/bash
# Round 5, check 2: check 1 (the whole GPU suite, the default bench line), then the A/B of the
# business grouping (r05_ab1.sh).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R || exit 1
bash profiles/scripts/r05_check1.sh || exit 1
bash profiles/scripts/r05_ab1.sh
