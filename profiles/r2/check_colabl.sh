#!/bin/bash
# colstrip store-shape ablation (wrong layout): contiguous 1-KiB row runs vs phase-plane runs
O=gpurun_out/colabl; mkdir -p $O
timeout -k 10 300 bash profiles/ab.sh $O/ab 2 colbase colabl &&
python3 -c "
import json,glob
for v in ('colbase','colabl'):
    xs=[json.load(open(f)) for f in sorted(glob.glob('$O/ab/%s.*.json'%v))]
    print(v, 'colscan ms', [round(x['kernel_ms_per_launch']['colscan'],4) for x in xs])
"
