#!/bin/bash
# Round 4: one-frame launches at 16 waves with the speculative rounds
# (SC_SPEC16 build: no VGPR spill now) against the 12-wave default, and C2
# with either build (parity only if adopted).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/r4spec16; mkdir -p $O; cd $R
B="python3 bench.py --no-cpu --host-steps 0 --latency-steps 0 --warmup 3"
for r in 1 2 3; do
  for v in "cur:12" "cur:16" "spec16:16"; do
    lib=${v%%:*}; w=${v##*:}
    SURFCASCADE_LIB=$R/surfcascade_amd/lib/variants/$lib/libsurfcascade.so timeout -k 10 200 $B --batch 1 --steps 50 --opt chain_waves=$w \
      > $O/b1_${lib}_w$w.$r.json 2> $O/b1_${lib}_w$w.$r.err || exit 1
  done
  for lib in cur spec16; do
    SURFCASCADE_LIB=$R/surfcascade_amd/lib/variants/$lib/libsurfcascade.so timeout -k 10 200 $B --steps 10 \
      > $O/c2_$lib.$r.json 2> $O/c2_$lib.$r.err || exit 1
  done
done
python3 profiles/ab_report_kernels.py $O
