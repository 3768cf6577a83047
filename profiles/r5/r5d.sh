#!/bin/bash
# Round 5, fourth GPU call: an 8-wave chain kernel (fewer rows in flight per
# XCD) against the defaults on C4 / C2 and on C4's widest levels alone;
# one-frame sub-queue / block-size combinations.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=gpurun_out/r5d; mkdir -p $O
PYTEST_K="chain_waves or fused_integral" bash profiles/run.sh r5d "pytest" \
  "abopt c4 2 base: w8:chain_waves=8 -- --config C4" \
  "abopt c2 2 base: w8:chain_waves=8 w12:chain_waves=12" \
  "abopt b1 4 base: q8:chain_subq=8 q8rb4:chain_subq=8,row_order=3,row_block=4 rb4:row_order=3,row_block=4 -- --batch 1 --steps 50" || exit 1
for w in 12 8; do
  timeout -k 10 300 python3 profiles/level_split.py --ranges 0:24,24:32 --steps 3 --batch 8 --width 3840 --height 2160 \
    --levels 32 --opt chain_waves=$w > $O/split_c4_w$w.txt 2>&1 || exit 1
done
cat $O/split_c4_w*.txt | grep levels
echo done
