#!/bin/bash
# Round 4: the LDS-DMA item variant (itembench V15) against the production
# item (V0), its TD counters; and a C2 bench line read against the HEAD PMC table.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=gpurun_out/r4ib15; mkdir -p $R/$O; cd $R
bash profiles/run.sh r4ib15 "itembench --reps 5 --variants 0:12,15:12,0:8,15:8" "bench c2 --latency-steps 0" || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE SQ_LDS_IDX_ACTIVE --kernel-trace \
    --output-format csv -d $R/$O/td -o pmc -- python3 $R/profiles/itembench/run.py --reps 1 --variants 0:12,15:12 \
    > $R/$O/td.txt 2>&1 || exit 1
echo done
