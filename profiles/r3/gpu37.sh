#!/bin/bash
# Round 3, call 37: one-frame launches with a narrower segment 0 (10 / 15 /
# 20 % of each row; the other 3 segments share the rest), after parity.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g37
mkdir -p $O
cd $R
for v in p15; do
  SURFCASCADE_LIB=$R/surfcascade_amd/lib/variants/$v/libsurfcascade.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "segments or single or batch_equals or pedestrian or level_range" > $O/pytest_$v.txt 2>&1 || { tail -30 $O/pytest_$v.txt; exit 1; }
  tail -1 $O/pytest_$v.txt
done
bash profiles/ab.sh gpurun_out/r3g37/b1 3 cur p10 p15 p20 -- --batch 1 --steps 50 && python3 profiles/ab_report_kernels.py gpurun_out/r3g37/b1 > $O/b1.txt && cat $O/b1.txt
