#!/bin/bash
# Round 3: probe of the top-k dense counts on the business side (which sources' |H3| differ).
set -o pipefail
cd $GRAFT_REPO_ROOT || exit 1
timeout -k 10 300 python -u profiles/scripts/r03_topk_biz_probe.py
