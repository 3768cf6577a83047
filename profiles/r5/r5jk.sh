#!/bin/bash
# Round 5: r5j (16-row column blocks) and r5k (chain batch sizes) in one call.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
bash profiles/r5/r5j.sh && bash profiles/r5/r5k.sh
