#!/bin/bash
# rowcarry 8 strips of loads in flight vs base: repeat A/B (rowscan / colscan / windows ms per launch)
O=gpurun_out/rc2; mkdir -p $O
timeout -k 10 500 bash profiles/ab.sh $O/ab 4 rc8 base && python3 profiles/ab_report.py $O/ab &&
python3 -c "
import json,glob
for v in ('base','rc8'):
    xs=[json.load(open(f))['kernel_ms_per_launch'] for f in sorted(glob.glob('$O/ab/%s.*.json'%v))]
    print(v, 'rowscan ms', [round(x['rowscan'],4) for x in xs], 'colscan', [round(x['colscan'],4) for x in xs])
    print(v, 'step ms', [round(json.load(open(f))['ms_per_step'],3) for f in sorted(glob.glob('$O/ab/%s.*.json'%v))])
"
