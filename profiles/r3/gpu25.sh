#!/bin/bash
# Round 3, call 25: rowcarry with dword loads (rowcarry4) and 4-B host pitch:
# parity (integral tests, pitch / offset cases), then C2 and batch-1 A/B
# against the byte-load rowcarry.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g25
mkdir -p $O
cd $R
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_mine.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
bash profiles/ab.sh gpurun_out/r3g25/c2 2 byte cur && python3 profiles/ab_report_kernels.py gpurun_out/r3g25/c2 > $O/c2.txt && cat $O/c2.txt || exit 1
bash profiles/ab.sh gpurun_out/r3g25/b1 2 byte cur -- --batch 1 --steps 50 && python3 profiles/ab_report_kernels.py gpurun_out/r3g25/b1 > $O/b1.txt && cat $O/b1.txt
