#!/bin/bash
# Round 5: C5 (pedestrian model, 12 waves by its LDS) at 10 waves; the C2
# line with the leaner Python enqueue path and 5 colseg segments (one-frame
# latency leg); parity of the column-pass tests at 5 segments.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
PYTEST_K="integral or column_pass or one_frame or stream" bash profiles/run.sh r5i "pytest" \
  "abopt c5 2 base: w10:chain_waves=10 -- --config C5" "bench c2" || exit 1
echo done
