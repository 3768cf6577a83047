#!/bin/bash
# Round 3, call 36: launch fill (segment-s waves first take K*s/DEN segment-0
# tasks) re-measured with the speculative idle rounds: s/2 (cur), s, 2s, 4s.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g36
mkdir -p $O
cd $R
bash profiles/ab.sh gpurun_out/r3g36/b1 3 cur f1 f2 f4 -- --batch 1 --steps 50 && python3 profiles/ab_report_kernels.py gpurun_out/r3g36/b1 > $O/b1.txt && cat $O/b1.txt || exit 1
bash profiles/ab.sh gpurun_out/r3g36/c2 2 cur f1 f2 && python3 profiles/ab_report_kernels.py gpurun_out/r3g36/c2 > $O/c2.txt && cat $O/c2.txt
