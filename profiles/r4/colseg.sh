#!/bin/bash
# Round 4: one-frame column pass in row segments (colblock + colseg, exact
# start values from 32-row block sums): GPU suite on the 8-segment build, the
# integral tests on the 4-segment one, then the one-frame A/B.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
bash profiles/run.sh r4colseg8 "lib colseg8" "pytest" &&
bash profiles/run.sh r4colseg4 "lib colseg4" "pytest tests/test_gpu_parity.py" &&
bash profiles/run.sh r4colseg "ab b1 4 cur colseg4 colseg8 -- --batch 1 --steps 50"
