#!/bin/bash
# how much of the window kernel's beyond-L2 traffic reaches DRAM (vs Infinity-Cache hits)
O=gpurun_out/pmc_dram; R=$PWD; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --list-avail > $R/$O/avail.txt 2>&1
grep -o "TCC_EA0_[A-Z_]*\|TCC_EA_[A-Z_]*\|MALL[A-Z_]*\|TCC_BUBBLE[A-Z_]*" $R/$O/avail.txt | sort -u > $R/$O/ea_counters.txt
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum --kernel-trace --output-format csv -d $R/$O/p1 -o pmc -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --host-steps 0 --latency-steps 0 > $R/$O/p1.json 2> $R/$O/p1.err
echo rc=$?
