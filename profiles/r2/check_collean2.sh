#!/bin/bash
# register-lean colstrip at 1, 2 and 5 waves per SIMD (dynamic-LDS caps) vs base: colscan ms per launch
O=gpurun_out/collean2; mkdir -p $O
timeout -k 10 500 bash profiles/ab.sh $O/ab 2 base lean lean1 lean2 &&
python3 -c "
import json,glob
for v in ('base','lean','lean1','lean2'):
    xs=[json.load(open(f))['kernel_ms_per_launch'] for f in sorted(glob.glob('$O/ab/%s.*.json'%v))]
    print(v, 'colscan ms', [round(x['colscan'],4) for x in xs], 'rowscan', [round(x['rowscan'],4) for x in xs])
"
