#!/bin/bash
# Round 3, call 39: C4 (8 x 4K, 32 levels) schedule sweep: row block 16 / 64,
# 4 segments per row, 16 waves.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g39
mkdir -p $O
cd $R
bash profiles/ab_opts.sh gpurun_out/r3g39/c4 2 base: rb16:row_block=16 rb64:row_block=64 s4:chain_segs=4 w16:chain_waves=16 -- --config C4 && \
  python3 profiles/ab_report_kernels.py gpurun_out/r3g39/c4 > $O/c4.txt && cat $O/c4.txt
