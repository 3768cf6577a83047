#!/bin/bash
# Round 3, call 45: the row carries of fused frames computed by the chain
# kernel's walkers (rowcarry4 rows, write-through, per-frame counts):
# parity, then C2 A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g45
mkdir -p $O
cd $R
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
bash profiles/ab.sh gpurun_out/r3g45/c2 3 old cur && python3 profiles/ab_report_kernels.py gpurun_out/r3g45/c2 > $O/c2.txt && cat $O/c2.txt
