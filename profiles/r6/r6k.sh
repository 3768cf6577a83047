#!/bin/bash
# Round 6, call k: the task timeline of one rank of the single-frame split
# (profiling build, SC_PROF_CHAIN): rank 0 of W = 8 and the whole frame, 4 and
# 8 segments per row: where the ~0.2 ms every one-frame launch costs goes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6k; mkdir -p $O
export SURFCASCADE_LIB=$R/surfcascade_amd/lib/variants/prof/libsurfcascade.so
for w in 1 8; do for sg in 4 8; do
  timeout -k 10 200 python3 profiles/shard_balance.py --config C2 --worlds $w --steps 2 --opt profile=1 --opt chain_segs=$sg \
    > $O/w${w}_s$sg.txt 2> $O/w${w}_s$sg.err || exit 1
  echo "== W $w segs $sg"; grep "SC_PROF_WAVES\|SC_PROF_TASKS" $O/w${w}_s$sg.err | tail -$((sg + 1))
done; done
