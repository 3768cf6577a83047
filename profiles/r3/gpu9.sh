#!/bin/bash
# Round 3, call 9: colstrip occupancy variants (rows of loads in flight vs
# waves per SIMD), per-kernel times.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g9
mkdir -p $O
cd $R
V=${VARIANTS:-cur colu8 colu6 colu4}
bash profiles/ab.sh gpurun_out/r3g9/c2 3 $V && python3 profiles/ab_report_kernels.py gpurun_out/r3g9/c2 > $O/c2.txt && cat $O/c2.txt
