#!/bin/bash
# with the launch fill: segments per row at 32 frames per launch (8 default vs 4)
O=gpurun_out/segs32; mkdir -p $O
for r in 1 2; do
  for sg in 8 4; do
    timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu --latency-steps 0 --host-steps 0 --opt chain_segs=$sg > $O/s$sg.$r.json 2> $O/s$sg.$r.err || { tail -3 $O/s$sg.$r.err; exit 1; }
  done
done
python3 -c "
import json,glob
for sg in (8,4):
    xs=[json.load(open(f))['kernel_ms_per_launch']['windows'] for f in sorted(glob.glob('$O/s%d.*.json'%sg))]
    print(sg, [round(x,3) for x in xs])
"
