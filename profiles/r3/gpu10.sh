#!/bin/bash
# Round 3, call 10: fused integral (column walks inside the chain kernel):
# parity, then C2 A/B against the separate integral kernels.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g10
mkdir -p $O
cd $R
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "fused or integral_batch or batch_equals" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -3 $O/pytest.txt
bash profiles/ab_opts.sh gpurun_out/r3g10/c2 3 sep:integral_fuse=1 fuse:integral_fuse=0 pre2:integral_pre=2 && \
  python3 profiles/ab_report_kernels.py gpurun_out/r3g10/c2 > $O/c2.txt && cat $O/c2.txt
