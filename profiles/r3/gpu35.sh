#!/bin/bash
# Round 3, call 35: task trace of a one-frame launch and a 32-frame launch
# (SC_PROF_CHAIN build): per segment, the entry wait and evaluation times.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g35
mkdir -p $O
cd $R
export SURFCASCADE_LIB=$R/surfcascade_amd/lib/variants/prof/libsurfcascade.so
for b in 1 32; do
  timeout -k 10 200 python3 bench.py --steps 3 --warmup 0 --no-cpu --latency-steps 0 --host-steps 0 --batch $b --opt profile=1 > $O/p$b.json 2> $O/p$b.err || { tail -5 $O/p$b.err; exit 1; }
  grep "SC_PROF_WAVES\|SC_PROF_TASKS" $O/p$b.err | tail -10
done
