#!/bin/bash
# Round 3, call 42: colsum4 with 48 / 96 / 128 rows of loads in flight (one frame).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g42
mkdir -p $O
cd $R
bash profiles/ab.sh gpurun_out/r3g42/b1 3 cur a96 a128 -- --batch 1 --steps 50 && python3 profiles/ab_report_kernels.py gpurun_out/r3g42/b1 > $O/b1.txt && cat $O/b1.txt
