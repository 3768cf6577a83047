#!/bin/bash
# round-2 item-loop ablations (run on the GPU box from the repo root):
# variant 3 with --fold F folds every corner's table row into rows & F (an
# L2-resident band) -- same lanes->lines pattern, no beyond-L2 gathers
set -e
mkdir -p gpurun_out/ib
run() { n=$1; shift; timeout -k 10 150 python profiles/itembench/run.py --reps 5 "$@" > gpurun_out/ib/$n.txt 2>&1; grep -E "variant" gpurun_out/ib/$n.txt | sed "s/^/$n /"; }
run base --variants 0:12,3:12
run fold15 --variants 0:12,3:12,3:16 --fold 15
run fold63 --variants 0:12,3:12 --fold 63
run fold255 --variants 0:12,3:12 --fold 255
