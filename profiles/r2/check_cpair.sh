#!/bin/bash
# colstrip per channel pair (1920 waves): integral/grid parity tests, then A/B of colscan
O=gpurun_out/cpair; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 bash profiles/ab.sh $O/ab 3 base cpair && python3 profiles/ab_report.py $O/ab &&
python3 -c "
import json,glob
for v in ('base','cpair'):
    xs=[json.load(open(f)) for f in sorted(glob.glob('$O/ab/%s.*.json'%v))]
    print(v, 'colscan ms', [round(x['kernel_ms_per_launch']['colscan'],4) for x in xs], 'ms/step', [round(x['ms_per_step'],3) for x in xs])
"
