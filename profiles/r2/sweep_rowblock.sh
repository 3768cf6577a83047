#!/bin/bash
# chain-kernel row block (grid rows per queue block) at the 32-frame default, interleaved
O=gpurun_out/sweep_rb; mkdir -p $O
for r in 1 2; do
  for rb in 16 24 32 40 48; do
    timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu --latency-steps 0 --host-steps 0 --opt row_block=$rb > $O/rb$rb.$r.json 2> $O/rb$rb.$r.err || { tail -3 $O/rb$rb.$r.err; exit 1; }
  done
done
python3 -c "
import json,glob
for rb in (16,24,32,40,48):
    xs=[json.load(open(f))['kernel_ms_per_launch']['windows'] for f in sorted(glob.glob('$O/rb%d.*.json'%rb))]
    print(rb, [round(x,3) for x in xs])
"
