#!/bin/bash
# Round 3, call 55: one-frame fused column pass, walker speed: sc1 stores
# with 192-row bands, plain stores + release per band (profiling builds).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g55
mkdir -p $O
cd $R
for v in prof192 profp; do
  SURFCASCADE_LIB=$R/surfcascade_amd/lib/variants/$v/libsurfcascade.so timeout -k 10 200 python3 bench.py --batch 1 --steps 20 --warmup 3 --no-cpu --latency-steps 0 --host-steps 0 --opt profile=1 > $O/$v.json 2> $O/$v.err || { tail -5 $O/$v.err; exit 1; }
  echo "== $v"; grep "SC_PROF_WA\|seg 0" $O/$v.err | tail -3
done
