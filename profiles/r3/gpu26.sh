#!/bin/bash
# Round 3, call 26: fused walk loading each image row once (byte per lane +
# 2-lane halo, DPP neighbours, rolling rows, 16 rows in flight) vs HEAD.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g26
mkdir -p $O
cd $R
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
bash profiles/ab.sh gpurun_out/r3g26/c2 3 old cur && python3 profiles/ab_report_kernels.py gpurun_out/r3g26/c2 > $O/c2.txt && cat $O/c2.txt
