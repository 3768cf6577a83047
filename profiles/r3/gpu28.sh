#!/bin/bash
# Round 3, call 28: one-frame step: lazy chain kernel vs the full grid
# (cascade + walk kernels, no hand-offs), and 2 / 4 segments at 12 waves.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g28
mkdir -p $O
cd $R
bash profiles/ab_opts.sh gpurun_out/r3g28/b1 3 lazy: full:full_grid=1 -- --batch 1 --steps 50 && \
  python3 profiles/ab_report_kernels.py gpurun_out/r3g28/b1 > $O/b1.txt && cat $O/b1.txt
