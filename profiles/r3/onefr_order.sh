#!/bin/bash
# one-frame launches: chain task order (row_order 0 level-major, 1 y-major, 2 blocks) and row-block size
O=gpurun_out/onefr; mkdir -p $O
for r in 1 2; do
  for v in "2 32" "0 32" "1 32" "2 8" "2 128" "2 512"; do
    set -- $v
    timeout -k 10 200 python bench.py --batch 1 --steps 40 --warmup 5 --no-cpu --latency-steps 0 --host-steps 0 --opt row_order=$1 --opt row_block=$2 > $O/o$1_b$2.$r.json 2> $O/o$1_b$2.$r.err || exit 1
    python -c "import json;d=json.load(open('$O/o$1_b$2.$r.json'));print('order $1 block $2', round(d['ms_per_step'],4), {k:round(v,4) for k,v in d['kernel_ms_per_launch'].items()})"
  done
done
