#!/bin/bash
set -e
mkdir -p gpurun_out/ib
timeout -k 10 150 python profiles/itembench/run.py --reps 5 --variants 0:12,8:12,10:12,10:16,10:8 > gpurun_out/ib/uhalf.txt 2>&1
grep variant gpurun_out/ib/uhalf.txt
