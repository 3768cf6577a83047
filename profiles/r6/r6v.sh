#!/bin/bash
# Round 6, call v: the one-frame task timeline at the final defaults (one task
# per wave, 4 sub-queues; profiling build SC_PROF_CHAIN): per segment the
# entry wait and evaluation, and when the waves leave.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6v; mkdir -p $O
export SURFCASCADE_LIB=$R/surfcascade_amd/lib/variants/prof/libsurfcascade.so
for w in 1 8; do
  timeout -k 10 200 python3 profiles/shard_balance.py --config C2 --worlds $w --steps 2 --opt profile=1 \
    > $O/w${w}.txt 2> $O/w${w}.err || exit 1
  echo "== W $w"; grep "SC_PROF_WAVES\|SC_PROF_TASKS" $O/w${w}.err | tail -9
done
