#!/bin/bash
# Round 5: the chain kernel's windows per slot and round (kBatch 96 / 160 /
# 192 vs 128) at C2's 16 waves and one frame's 12, with parity on each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
for v in b96 b160 b192; do
  SURFCASCADE_LIB=$R/surfcascade_amd/lib/variants/$v/libsurfcascade.so PYTEST_K="chain_waves or speculative or fused_integral" \
    bash profiles/run.sh r5k_$v "pytest" || exit 1
done
bash profiles/run.sh r5k "ab c2 2 cur b96 b160 b192" "ab b1 3 cur b96 b160 -- --batch 1 --steps 50" || exit 1
echo done
