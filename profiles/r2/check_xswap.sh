#!/bin/bash
# permlane32_swap semantics probe, then the paired-half load variant (V12) in the item microbenchmark
O=gpurun_out/xswap; mkdir -p $O
timeout -k 10 60 ./profiles/itembench/permlane_probe > $O/probe.txt 2>&1; cat $O/probe.txt
timeout -k 10 200 python profiles/itembench/run.py --reps 5 --variants 0:12,12:12,13:12,13:16,0:12,13:12 > $O/ib.txt 2>&1; rc=$?
grep variant $O/ib.txt; tail -3 $O/ib.txt; exit $rc
