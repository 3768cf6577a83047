#!/bin/bash
# Round 5: hand-off polls through the scalar path (SC_SPOLL 1: s_load glc of the
# entry / walk-count words, off the texture data path) vs the one-lane vector
# poll; parity on the variant, C2 / one frame / C4 A/B, C2 counters.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
SURFCASCADE_LIB=$R/surfcascade_amd/lib/variants/spoll/libsurfcascade.so \
  PYTEST_K="chain_waves or fused or c2_bench_form or one_frame or speculative or subq or shard" \
  bash profiles/run.sh r5l_spoll "pytest" || exit 1
bash profiles/run.sh r5l "ab c2 3 cur spoll" "ab b1 3 cur spoll -- --batch 1 --steps 50" \
  "ab c4 2 cur spoll -- --config C4" "lib spoll" "pmc pmc_spoll --config C2" || exit 1
echo done
