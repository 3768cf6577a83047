#!/bin/bash
# Round 5, fourth GPU call: (1) the one-frame column-block sums computed from
# the pixels inside rowcarry4's launch (colblock's launch and its R-row read
# gone): parity, A/B against the previous path (variant old) and with 6 / 8
# colseg segments; (2) an 8-wave chain kernel (fewer rows in flight per XCD)
# on C4 / C2 and on C4's widest levels alone; (3) one-frame sub-queue /
# block-size combinations.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
O=gpurun_out/r5e; mkdir -p $O
PYTEST_K="integral or one_frame or column_pass or segments or chain_waves or fused_integral or single" \
  bash profiles/run.sh r5e "pytest" \
  "ab ib1 4 old seg6 seg8 -- --batch 1 --steps 50" \
  "abopt b1 4 base: q8:chain_subq=8 q8rb4:chain_subq=8,row_order=3,row_block=4 rb4:row_order=3,row_block=4 -- --batch 1 --steps 50" \
  "abopt c4 2 base: w8:chain_waves=8 -- --config C4" \
  "abopt c2 2 base: w8:chain_waves=8" || exit 1
for w in 12 8; do
  timeout -k 10 300 python3 profiles/level_split.py --ranges 0:24,24:32 --steps 3 --batch 8 --width 3840 --height 2160 \
    --levels 32 --opt chain_waves=$w > $O/split_c4_w$w.txt 2>&1 || exit 1
done
grep levels $O/split_c4_w*.txt
echo done
