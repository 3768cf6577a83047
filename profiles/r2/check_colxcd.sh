#!/bin/bash
# XCD-aware colstrip block order: integral parity, then A/B (colscan ms per launch) vs base
O=gpurun_out/colxcd; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k integral -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 bash profiles/ab.sh $O/ab 3 base xcd && python3 profiles/ab_report.py $O/ab &&
python3 -c "
import json,glob
for v in ('base','xcd'):
    xs=[json.load(open(f))['kernel_ms_per_launch'] for f in sorted(glob.glob('$O/ab/%s.*.json'%v))]
    print(v, 'colscan ms', [round(x['colscan'],4) for x in xs], 'rowscan', [round(x['rowscan'],4) for x in xs])
"
