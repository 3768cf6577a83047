#!/bin/bash
# Round 3, call 18: fused integral with walkers in every 1st / 2nd / 4th / 8th
# workgroup (256 / 128 / 64 / 32 walking waves), C2.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g18
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "fused" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
bash profiles/ab.sh gpurun_out/r3g18/c2 3 w1 w2 w4 w8 && \
  python3 profiles/ab_report_kernels.py gpurun_out/r3g18/c2 > $O/c2.txt && cat $O/c2.txt
