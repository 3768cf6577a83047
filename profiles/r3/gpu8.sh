#!/bin/bash
# Round 3, call 8: parity suite on the current product build, then an A/B of
# chain-kernel variants on C2 (and C4 for the first two).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g8
mkdir -p $O
cd $R
echo "pytest" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
V=${VARIANTS:-cur mbits s1 b64 s3b64}
bash profiles/ab.sh gpurun_out/r3g8/c2 3 $V && python3 profiles/ab_report.py gpurun_out/r3g8/c2 > $O/c2.txt && cat $O/c2.txt
