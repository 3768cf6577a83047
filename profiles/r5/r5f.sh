#!/bin/bash
# Round 5, fifth GPU call: the full GPU suite on the new defaults (one-frame
# blocks of 4, C4 at 8 waves, block sums from the pixels inside rowcarry4's
# launch), the merged launch's waves per workgroup (cb4 / cb8 / cb16)
# against the previous path (old), 10 / 14 chain waves on C4 / C2, and the
# C2 / C4 lines.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
bash profiles/run.sh r5f "pytest" \
  "ab ib1 4 old cb4 cb8 cb16 -- --batch 1 --steps 50" \
  "abopt c4 2 base: w10:chain_waves=10 w12:chain_waves=12 -- --config C4" \
  "abopt c2 2 base: w14:chain_waves=14" \
  "bench c2" "bench c4 --config C4" || exit 1
echo done
