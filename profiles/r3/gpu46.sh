#!/bin/bash
# Round 3, call 46: debug the fused row carries (6 frames, pre 1, 12 / 16 waves).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g46
mkdir -p $O
cd $R
timeout -k 10 150 python3 -u profiles/r3/dbg_rcfuse.py 2>&1 | tee $O/dbg.txt
