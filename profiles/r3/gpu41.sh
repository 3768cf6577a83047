#!/bin/bash
# Round 3, call 41: rowcarry4 writes the R rows of the two-pass frames
# (rowfull skipped): integral parity, then one-frame and C2 A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g41
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "integral or fused or single or batch" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
bash profiles/ab.sh gpurun_out/r3g41/b1 3 old cur -- --batch 1 --steps 50 && python3 profiles/ab_report_kernels.py gpurun_out/r3g41/b1 > $O/b1.txt && cat $O/b1.txt || exit 1
bash profiles/ab.sh gpurun_out/r3g41/c2 2 old cur && python3 profiles/ab_report_kernels.py gpurun_out/r3g41/c2 > $O/c2.txt && cat $O/c2.txt
