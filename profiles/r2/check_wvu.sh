#!/bin/bash
# uniform wave index (per-wave LDS bases in SGPRs: 168 -> 153 VGPRs, no scratch): gpu suite + A/B
O=gpurun_out/wvu; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 bash profiles/ab.sh $O/ab 3 base wvu && python3 profiles/ab_report.py $O/ab
