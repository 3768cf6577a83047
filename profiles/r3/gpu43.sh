#!/bin/bash
# Round 3, call 43: one-frame launches: a lone active slot's free descriptor
# evaluates the other parity of its next windows; parity, then A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g43
mkdir -p $O
cd $R
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
bash profiles/ab.sh gpurun_out/r3g43/b1 3 old cur -- --batch 1 --steps 50 && python3 profiles/ab_report_kernels.py gpurun_out/r3g43/b1 > $O/b1.txt && cat $O/b1.txt
