#!/bin/bash
# Round 3, call 33: speculative idle rounds in the 16-wave kernel too (2 VGPR spills) at C2.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g33
mkdir -p $O
cd $R
bash profiles/ab.sh gpurun_out/r3g33/c2 3 cur sp16 && python3 profiles/ab_report_kernels.py gpurun_out/r3g33/c2 > $O/c2.txt && cat $O/c2.txt
