#!/bin/bash
# round-2 item-loop ablations (run on the GPU box from the repo root)
set -e
mkdir -p gpurun_out/ib
run() { n=$1; shift; timeout -k 10 150 python profiles/itembench/run.py --reps 5 "$@" > gpurun_out/ib/$n.txt 2>&1; grep -E "variant" gpurun_out/ib/$n.txt | sed "s/^/$n /"; }
run base --variants 0:12,3:12,0:16
run fold15 --variants 0:12,3:12,3:16 --omask 15
run fold63 --variants 0:12,3:12 --omask 63
run bcast0 --variants 0:12,2:12 --omask 0
