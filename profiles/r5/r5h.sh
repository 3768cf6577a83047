#!/bin/bash
# Round 5: one-frame integral variants -- the block role's neighbour bytes
# through the scalar cache (sb), 3 / 5 colseg segments -- against the default
# (r8), with their parity (integral / column-pass tests on each library).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
for v in sb seg3 seg5; do
  SURFCASCADE_LIB=$R/surfcascade_amd/lib/variants/$v/libsurfcascade.so PYTEST_K="integral or column_pass or one_frame" \
    bash profiles/run.sh r5h_$v "pytest" || exit 1
done
bash profiles/run.sh r5h "ab ib1 5 r8 sb seg3 seg5 -- --batch 1 --steps 50" || exit 1
echo done
