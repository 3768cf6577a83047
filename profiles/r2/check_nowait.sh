#!/bin/bash
# cost of the segment hand-off chain (timing ablation, wrong results) + phase counters
O=gpurun_out/nowait; mkdir -p $O
timeout -k 10 300 bash profiles/ab.sh $O/ab 3 base nowait && python3 profiles/ab_report.py $O/ab || exit 1
SURFCASCADE_LIB=$PWD/surfcascade_amd/lib/variants/prof/libsurfcascade.so timeout -k 10 120 \
  python3 bench.py --steps 1 --warmup 0 --no-cpu --latency-steps 0 --host-steps 0 --opt profile=1 > $O/prof.json 2> $O/prof.err
grep SC_PROF $O/prof.err | tail -1
