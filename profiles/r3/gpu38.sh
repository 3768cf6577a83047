#!/bin/bash
# Round 3, call 38: walker issue priority 0 / 2 (cur) / 3 at C2; fused parity tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g38
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "fused" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
bash profiles/ab.sh gpurun_out/r3g38/c2 3 cur pr0 pr3 && python3 profiles/ab_report_kernels.py gpurun_out/r3g38/c2 > $O/c2.txt && cat $O/c2.txt
