#!/bin/bash
# colstrip with non-temporal table stores: integral parity, A/B colscan / windows vs base
O=gpurun_out/colnt; mkdir -p $O
SURFCASCADE_LIB=$PWD/surfcascade_amd/lib/variants/nt/libsurfcascade.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "integral or batch" -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 bash profiles/ab.sh $O/ab 3 base nt && python3 profiles/ab_report.py $O/ab &&
python3 -c "
import json,glob
for v in ('base','nt'):
    xs=[json.load(open(f)) for f in sorted(glob.glob('$O/ab/%s.*.json'%v))]
    print(v, 'colscan', [round(x['kernel_ms_per_launch']['colscan'],4) for x in xs], 'windows', [round(x['kernel_ms_per_launch']['windows'],3) for x in xs])
"
