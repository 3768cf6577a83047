#!/bin/bash
# Round 5: one-frame launches whose two XCDs per segment take contiguous
# halves of the row list (SC_SPLIT_PARTS) instead of alternate tasks:
# parity of the one-frame / speculation / sub-queue / shard tests, A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
SURFCASCADE_LIB=$R/surfcascade_amd/lib/variants/split/libsurfcascade.so \
  PYTEST_K="one_frame or speculative or subq or batch1 or single or shard or segments or random_geometry or random_schedule" \
  bash profiles/run.sh r5split "pytest" || exit 1
bash profiles/run.sh r5split "ab b1 3 cur split -- --batch 1 --steps 50" || exit 1
echo done
