#!/bin/bash
# with the launch-fill default (s/2 segment-0 tasks per wave): segments per row at one frame per launch
O=gpurun_out/fill_segs; mkdir -p $O
for r in 1 2 3; do
  for sg in 4 8 2; do
    timeout -k 10 200 python3 bench.py --batch 1 --steps 20 --warmup 3 --no-cpu --latency-steps 0 --host-steps 0 --opt chain_segs=$sg > $O/s$sg.$r.json 2> $O/s$sg.$r.err || { tail -3 $O/s$sg.$r.err; exit 1; }
  done
done
python3 -c "
import json,glob
for sg in (4,8,2):
    xs=[json.load(open(f))['kernel_ms_per_launch']['windows'] for f in sorted(glob.glob('$O/s%d.*.json'%sg))]
    print(sg, [round(x,4) for x in xs])
"
