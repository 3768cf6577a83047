#!/bin/bash
# chain-kernel ms per frame against frames per launch (launch overhead = fill + drain), with the launch fill
O=gpurun_out/batch_curve; mkdir -p $O
for r in 1 2; do
  for b in 8 16 32 64; do
    timeout -k 10 200 python3 bench.py --batch $b --steps 8 --warmup 2 --no-cpu --latency-steps 0 --host-steps 0 > $O/b$b.$r.json 2> $O/b$b.$r.err || { tail -3 $O/b$b.$r.err; exit 1; }
  done
done
python3 -c "
import json,glob
for b in (8,16,32,64):
    xs=[json.load(open(f))['kernel_ms_per_launch']['windows']/b for f in sorted(glob.glob('$O/b%d.*.json'%b))]
    print(b, [round(x,4) for x in xs])
"
