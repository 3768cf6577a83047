#!/bin/bash
# Round 3, call 2: the GPU parity suite on the current library, then an
# interleaved A/B of chain-kernel variants (profiles/build_variants.sh).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g2
mkdir -p $O
cd $R
echo "calib" && (cd /tmp && timeout -k 10 120 $R/profiles/calib/fetch_calib > $O/calib.json 2> $O/calib.err) &&
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum --kernel-trace --output-format csv -d $O/calpmc -o pmc -- $R/profiles/calib/fetch_calib > $O/calpmc.log 2>&1) &&
echo "pytest" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
echo "ab" && bash profiles/ab.sh gpurun_out/r3g2/ab 3 ${VARIANTS:-base remat remat16} &&
python3 profiles/ab_report.py gpurun_out/r3g2/ab > $O/ab_report.txt 2>&1; cat $O/ab_report.txt
