#!/bin/bash
# Round 3, call 54: profiling build (phase counters, wave timeline, task
# trace, walker completion) of one-frame launches, fused column pass vs
# separate.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g54
mkdir -p $O
cd $R
for v in sep fused; do
  X="--opt profile=1"; [ $v == sep ] && X="$X --opt integral_fuse=1"
  SURFCASCADE_LIB=$R/surfcascade_amd/lib/variants/prof/libsurfcascade.so timeout -k 10 200 python3 bench.py --batch 1 --steps 20 --warmup 3 --no-cpu --latency-steps 0 --host-steps 0 $X > $O/$v.json 2> $O/$v.err || { tail -5 $O/$v.err; exit 1; }
  echo "== $v"; grep SC_PROF $O/$v.err | tail -8
done
