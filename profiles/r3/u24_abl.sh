#!/bin/bash
# u24 timing ablation: packed gathers without the unpack (wrong values) vs with, fusion off
O=gpurun_out/u24abl; mkdir -p $O
for r in 1 2; do
  for v in base:1 pad:1 base:2; do
    n=${v%%:*}; u=${v#*:}
    SURFCASCADE_LIB=$PWD/surfcascade_amd/lib/variants/$n/libsurfcascade.so timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu --latency-steps 0 --host-steps 0 --opt integral_fuse=1 --opt table_u24=$u > $O/$n.$u.$r.json 2> $O/$n.$u.$r.err || exit 1
    python -c "import json;d=json.load(open('$O/$n.$u.$r.json'));print('$n u24=$u', round(d['ms_per_step'],3), d['kernel_ms_per_launch']['windows'])"
  done
done
