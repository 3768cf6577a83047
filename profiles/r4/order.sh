#!/bin/bash
# Round 4: one-frame task order: the row blocks bottom-up (row_order 3: the
# last block dealt holds every level's top rows, the short rows of the wide
# levels last), interleaved against the default blocks top-down.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && bash profiles/run.sh r4order "abopt b1 3 o2:row_order=2 o3:row_order=3 o3b16:row_order=3,row_block=16 o2b8:row_order=2,row_block=8 o3b8:row_order=3,row_block=8 -- --batch 1 --steps 50" \
  "abopt c2 2 o2:row_order=2 o3:row_order=3" || exit 1
cd $R && timeout -k 10 120 python3 profiles/r4/synccost.py > gpurun_out/r4order/synccost.json 2> gpurun_out/r4order/synccost.err && cat gpurun_out/r4order/synccost.json
