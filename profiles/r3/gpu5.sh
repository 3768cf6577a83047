#!/bin/bash
# Round 3, call 5: A/B of chain-kernel variants (build_variants.sh), C2 and C4
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g5
mkdir -p $O
cd $R
V=${VARIANTS:-prev cur}
bash profiles/ab.sh gpurun_out/r3g5/c2 3 $V && python3 profiles/ab_report.py gpurun_out/r3g5/c2 > $O/c2.txt && cat $O/c2.txt &&
bash profiles/ab.sh gpurun_out/r3g5/c4 2 $V -- --config C4 && python3 profiles/ab_report.py gpurun_out/r3g5/c4 > $O/c4.txt && cat $O/c4.txt
