#!/bin/bash
# Round 4: one-frame call overhead legs (synccost.py), then the TLB counters.
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out/r4order; cd $R
timeout -k 10 120 python3 profiles/r4/synccost.py > gpurun_out/r4order/synccost.json 2> gpurun_out/r4order/synccost.err || { tail -5 gpurun_out/r4order/synccost.err; exit 1; }
cat gpurun_out/r4order/synccost.json
bash profiles/r4/tlb.sh
