#!/bin/bash
# Round 5, third GPU call: (1) the chain kernel's counters per level group
# (C2 levels 0-12 / 13-23, C4 levels 0-23 / 24-31: VERDICT r4 next #3);
# (2) the one-frame launch's timeline and per-segment task trace (profiling
# build); (3) one-frame sub-queues 4 vs 8 and bottom-up block sizes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=gpurun_out/r5c; mkdir -p $O
for rg in 0:13 13:24; do
  timeout -k 10 600 bash profiles/r5/level_pmc.sh $O/lvl_c2 $rg || exit 1
done
for rg in 0:24 24:32; do
  timeout -k 10 600 bash profiles/r5/level_pmc.sh $O/lvl_c4 $rg --batch 8 --width 3840 --height 2160 --levels 32 || exit 1
done
echo "level pmc done"
bash profiles/run.sh r5c "lib prof" \
  "bench prof_b1 --steps 5 --warmup 1 --no-cpu --latency-steps 0 --host-steps 0 --batch 1 --opt profile=1" || exit 1
unset SURFCASCADE_LIB
bash profiles/run.sh r5c "abopt b1 4 base: q8:chain_subq=8 rb4:row_order=3,row_block=4 rb12:row_order=3,row_block=12 -- --batch 1 --steps 50" || exit 1
echo done
