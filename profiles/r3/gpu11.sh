#!/bin/bash
# Round 3, call 11: fused-integral ablations (walk stores: sc1 / plain + release
# fence / none; walk queues global or per XCD), all with 2 frames integrated ahead.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g11
mkdir -p $O
cd $R
bash profiles/ab.sh gpurun_out/r3g11/c2 2 cur nost plain plainx sc1x -- --opt integral_pre=2 && \
  SURFCASCADE_LIB=$R/surfcascade_amd/lib/variants/cur/libsurfcascade.so bash profiles/ab_opts.sh gpurun_out/r3g11/c2 2 sep:integral_fuse=1 && \
  python3 profiles/ab_report_kernels.py gpurun_out/r3g11/c2 > $O/c2.txt && cat $O/c2.txt
