#!/bin/bash
# colstrip with two columns per lane: integral parity, then A/B (colscan ms per launch) vs base
O=gpurun_out/colpair; mkdir -p $O
SURFCASCADE_LIB=$PWD/surfcascade_amd/lib/variants/pair/libsurfcascade.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 bash profiles/ab.sh $O/ab 3 base pair pair4 && python3 profiles/ab_report.py $O/ab &&
python3 -c "
import json,glob
for v in ('base','pair','pair4'):
    xs=[json.load(open(f))['kernel_ms_per_launch'] for f in sorted(glob.glob('$O/ab/%s.*.json'%v))]
    print(v, 'colscan ms', [round(x['colscan'],4) for x in xs], 'rowscan', [round(x['rowscan'],4) for x in xs])
"
