#!/bin/bash
# readiness of freshly dequeued own tasks (first poll) and steals: profiling builds
O=gpurun_out/steal; mkdir -p $O
for v in trk stlp; do
SURFCASCADE_LIB=$PWD/surfcascade_amd/lib/variants/$v/libsurfcascade.so timeout -k 10 120 \
  python3 bench.py --steps 1 --warmup 0 --no-cpu --latency-steps 0 --host-steps 0 --opt profile=1 > $O/prof_$v.json 2> $O/prof_$v.err || exit 1
echo $v; grep SC_PROF $O/prof_$v.err | tail -1
done
