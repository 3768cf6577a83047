#!/bin/bash
# Round 3, call 12: (a) fused-walk cost without its stores (tables prebuilt by
# the separate kernels, walks run and signal but store nothing); (b) batch-1
# step options: segments per row and chain-kernel width.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g12
mkdir -p $O
cd $R
bash profiles/ab.sh gpurun_out/r3g12/c2 2 cur nost -- --opt integral_pre=2 && \
  python3 profiles/ab_report_kernels.py gpurun_out/r3g12/c2 > $O/c2.txt && cat $O/c2.txt && \
SURFCASCADE_LIB=$R/surfcascade_amd/lib/variants/cur/libsurfcascade.so bash profiles/ab_opts.sh gpurun_out/r3g12/b1 2 \
  s4w16: s1:chain_segs=1 s2:chain_segs=2 s8:chain_segs=8 s4w12:chain_waves=12 s2w12:chain_segs=2,chain_waves=12 -- --batch 1 --steps 50 && \
  python3 profiles/ab_report_kernels.py gpurun_out/r3g12/b1 > $O/b1.txt && cat $O/b1.txt
