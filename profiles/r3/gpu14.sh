#!/bin/bash
# Round 3, call 14: rowcarry with 1 / 2 / 4 / 8 rows (waves) per workgroup, C2 and batch 1.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g14
mkdir -p $O
cd $R
bash profiles/ab.sh gpurun_out/r3g14/c2 2 cur r2 r4 r8 && \
  python3 profiles/ab_report_kernels.py gpurun_out/r3g14/c2 > $O/c2.txt && cat $O/c2.txt && \
bash profiles/ab.sh gpurun_out/r3g14/b1 2 cur r2 r4 r8 -- --batch 1 --steps 50 && \
  python3 profiles/ab_report_kernels.py gpurun_out/r3g14/b1 > $O/b1.txt && cat $O/b1.txt
