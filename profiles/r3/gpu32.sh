#!/bin/bash
# Round 3, call 32: C5 (380-weak pedestrian model) at 16 waves with the
# weights read through the caches vs 12 waves with the weights in LDS.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g32
mkdir -p $O
cd $R
bash profiles/ab_opts.sh gpurun_out/r3g32/c5 2 w12: w16:chain_waves=16 w12c:lds_weights=0 -- --config C5 && \
  python3 profiles/ab_report_kernels.py gpurun_out/r3g32/c5 > $O/c5.txt && cat $O/c5.txt
