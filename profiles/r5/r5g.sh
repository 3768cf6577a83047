#!/bin/bash
# Round 5: the merged launch's block role with 8 / 16 image rows of loads in
# flight (one frame), parity of the C4 forms at 10 waves and of the integral
# paths, the C4 line at 10 waves.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
PYTEST_K="c4 or integral or column_pass or one_frame or chain_waves" bash profiles/run.sh r5g "pytest" \
  "ab ib1 4 r8 r16 -- --batch 1 --steps 50" "bench c4 --config C4 --latency-steps 0" || exit 1
echo done
