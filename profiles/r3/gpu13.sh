#!/bin/bash
# Round 3, call 13: full GPU suite on the fused-integral defaults, then
# rowcarry with 4 / 8 / 16 strips of loads in flight (C2 A/B).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g13
mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -3 $O/pytest.txt
bash profiles/ab.sh gpurun_out/r3g13/c2 2 cur rc8 rc16 && \
  python3 profiles/ab_report_kernels.py gpurun_out/r3g13/c2 > $O/c2.txt && cat $O/c2.txt
