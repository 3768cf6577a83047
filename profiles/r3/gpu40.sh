#!/bin/bash
# Round 3, call 40: speculative idle rounds limited to one-frame launches:
# C4, C5 and one-frame checks.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g40
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "constant or single or segments or fused" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
bash profiles/ab.sh gpurun_out/r3g40/c4 2 cur -- --config C4 && python3 profiles/ab_report_kernels.py gpurun_out/r3g40/c4 > $O/c4.txt && cat $O/c4.txt || exit 1
bash profiles/ab.sh gpurun_out/r3g40/b1 2 cur -- --batch 1 --steps 50 && python3 profiles/ab_report_kernels.py gpurun_out/r3g40/b1 > $O/b1.txt && cat $O/b1.txt || exit 1
bash profiles/ab.sh gpurun_out/r3g40/c5 2 cur -- --config C5 && python3 profiles/ab_report_kernels.py gpurun_out/r3g40/c5 > $O/c5.txt && cat $O/c5.txt
