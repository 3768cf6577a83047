#!/bin/bash
# Round 4: deferred late stages -- the GPU suite on the product build, then
# interleaved A/B of the chain kernel with / without deferral (C2, one
# frame, C5) and two flush thresholds.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=gpurun_out/r4defer; mkdir -p $R/$O; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
bash profiles/ab.sh $O/c2 3 nodefer defer q64f16 q64f48 || exit 1
python3 profiles/ab_report.py $O/c2
bash profiles/ab.sh $O/b1 3 nodefer defer -- --batch 1 --steps 40 || exit 1
python3 profiles/ab_report.py $O/b1
bash profiles/ab.sh $O/c5 2 nodefer defer -- --config C5 || exit 1
python3 profiles/ab_report.py $O/c5
