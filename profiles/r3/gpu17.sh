#!/bin/bash
# Round 3, call 17: visited counts summed per wave (one atomic per wave, not
# per task; 16-wave kernel without VGPR spills) vs the previous commit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g17
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
bash profiles/ab.sh gpurun_out/r3g17/c2 3 old cur && \
  python3 profiles/ab_report_kernels.py gpurun_out/r3g17/c2 > $O/c2.txt && cat $O/c2.txt && \
bash profiles/ab.sh gpurun_out/r3g17/b1 2 old cur -- --batch 1 --steps 50 && \
  python3 profiles/ab_report_kernels.py gpurun_out/r3g17/b1 > $O/b1.txt && cat $O/b1.txt
