#!/bin/bash
# round-2 item-loop variants: 4 = two lanes per item on interleaved cells;
# 5/6/7 = arithmetic ablations (no Normalize / f32 sigmoid / both)
set -e
mkdir -p gpurun_out/ib
run() { n=$1; shift; timeout -k 10 150 python profiles/itembench/run.py --reps 5 "$@" > gpurun_out/ib/$n.txt 2>&1; grep -E "variant" gpurun_out/ib/$n.txt | sed "s/^/$n /"; }
run pair --variants 0:12,4:12,4:8,4:16,5:12,6:12,7:12
