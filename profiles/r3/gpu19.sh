#!/bin/bash
# Round 3, call 19: fused integral with 1 or 2 walking waves per workgroup; 2 or 3 frames integrated ahead.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g19
mkdir -p $O
cd $R
bash profiles/ab.sh gpurun_out/r3g19/c2 3 w1 w2pw && \
  SURFCASCADE_LIB=$R/surfcascade_amd/lib/variants/w1/libsurfcascade.so bash profiles/ab_opts.sh gpurun_out/r3g19/c2 3 pre3:integral_pre=3 && \
  python3 profiles/ab_report_kernels.py gpurun_out/r3g19/c2 > $O/c2.txt && cat $O/c2.txt
