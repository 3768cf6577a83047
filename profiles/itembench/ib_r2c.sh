#!/bin/bash
# uniform corner loads (variant 8) vs the production item (0); PMC of both
set -e
mkdir -p gpurun_out/ib
timeout -k 10 150 python profiles/itembench/run.py --reps 5 --variants 0:12,8:12,8:8,4:16 > gpurun_out/ib/uload.txt 2>&1
grep variant gpurun_out/ib/uload.txt
V=0:12,8:12 bash profiles/itembench/ib_pmc.sh
