#!/bin/bash
# Round 3, call 27: chain-kernel phase counters (SC_PROF_CHAIN build) at
# batch 1 and batch 32 (C2): where a one-frame launch's time goes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g27
mkdir -p $O
cd $R
export SURFCASCADE_LIB=$R/surfcascade_amd/lib/variants/prof/libsurfcascade.so
for b in 1 32; do
  timeout -k 10 200 python3 bench.py --steps 10 --warmup 0 --no-cpu --latency-steps 0 --host-steps 0 --batch $b --opt profile=1 > $O/b$b.json 2> $O/b$b.err || { tail -5 $O/b$b.err; exit 1; }
  grep SC_PROF_CHAIN $O/b$b.err | tail -1
done
