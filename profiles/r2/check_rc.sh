#!/bin/bash
# rowcarry: strips of pixel loads in flight (4 base, 8, 12): integral parity with each, A/B rowscan ms per launch
O=gpurun_out/rc; mkdir -p $O
for v in rc8 rc12; do
SURFCASCADE_LIB=$PWD/surfcascade_amd/lib/variants/$v/libsurfcascade.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k integral -x -q --timeout 120 --timeout-method thread > $O/pytest_$v.log 2>&1 || { tail -5 $O/pytest_$v.log; exit 1; }
tail -1 $O/pytest_$v.log
done
timeout -k 10 500 bash profiles/ab.sh $O/ab 3 base rc8 rc12 &&
python3 -c "
import json,glob
for v in ('base','rc8','rc12'):
    xs=[json.load(open(f))['kernel_ms_per_launch'] for f in sorted(glob.glob('$O/ab/%s.*.json'%v))]
    print(v, 'rowscan ms', [round(x['rowscan'],4) for x in xs], 'colscan', [round(x['colscan'],4) for x in xs])
"
