#!/bin/bash
set -e
mkdir -p gpurun_out/ib
timeout -k 10 150 python profiles/itembench/run.py --reps 5 --variants 0:12,8:12,9:12,9:16,9:8 > gpurun_out/ib/pairu.txt 2>&1
grep variant gpurun_out/ib/pairu.txt
ONLY1=1 V=8:12,9:16 bash profiles/itembench/ib_pmc.sh
