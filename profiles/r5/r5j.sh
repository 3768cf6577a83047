#!/bin/bash
# Round 5: the one-frame column pass with 16-row blocks (the merged launch's
# block role walks half the rows; colseg sums twice as many block values),
# with 5 and 6 segments, against the default 32-row blocks (cur).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
for v in blk16 blk16s6; do
  SURFCASCADE_LIB=$R/surfcascade_amd/lib/variants/$v/libsurfcascade.so PYTEST_K="integral or column_pass or one_frame" \
    bash profiles/run.sh r5j_$v "pytest" || exit 1
done
bash profiles/run.sh r5j "ab ib1 5 cur blk16 blk16s6 -- --batch 1 --steps 50" || exit 1
echo done
