#!/bin/bash
# integral form by frames per launch with the per-channel colsum: colstrip (1) vs rowfull + colsum (2)
O=gpurun_out/passes; mkdir -p $O
for r in 1 2; do
  for b in 2 3 4 6 8; do
    for p in 1 2; do
      timeout -k 10 200 python3 bench.py --batch $b --steps 10 --warmup 2 --no-cpu --latency-steps 0 --host-steps 0 --opt integral_passes=$p > $O/b$b.p$p.$r.json 2> $O/b$b.p$p.$r.err || { tail -3 $O/b$b.p$p.$r.err; exit 1; }
    done
  done
done
python3 -c "
import json,glob
for b in (2,3,4,6,8):
    for p in (1,2):
        xs=[json.load(open(f))['kernel_ms_per_launch'] for f in sorted(glob.glob('$O/b%d.p%d.*.json'%(b,p)))]
        print(b, p, [round(x['colscan']+x['rowscan'],4) for x in xs])
"
