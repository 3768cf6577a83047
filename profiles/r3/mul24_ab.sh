#!/bin/bash
# A/B: per-item column math with 24-bit multiplies (mul24) vs quarter-rate 32-bit (base)
O=gpurun_out/mul24; mkdir -p $O
for r in 1 2 3; do
  for v in base mul24; do
    SURFCASCADE_LIB=$PWD/surfcascade_amd/lib/variants/$v/libsurfcascade.so timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --latency-steps 10 --host-steps 0 > $O/$v.$r.json 2> $O/$v.$r.err || exit 1
    python -c "import json;d=json.load(open('$O/$v.$r.json'));print('$v', round(d['ms_per_step'],3), round(d['kernel_ms_per_launch']['windows'],3), round(d['latency_batch1']['ms_per_frame'],4))"
  done
done
