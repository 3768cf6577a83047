#!/bin/bash
# Round 3, first GPU call: baseline bench, level-group split, FETCH_SIZE
# calibration (profiles/calib), with PMC passes.  Run from the repo root.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
echo "calib plain" && timeout -k 10 120 $R/profiles/calib/fetch_calib > $O/calib.json 2> $O/calib.err &&
pmc() { local n=$1; shift; timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $O/$n -o pmc -- $R/profiles/calib/fetch_calib > $O/$n.log 2>&1; }
echo "calib pmc" && pmc cf FETCH_SIZE && pmc cw WRITE_SIZE && pmc ct TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum &&
pmc cl TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE &&
echo "bench" && timeout -k 10 300 python3 $R/bench.py --cpu-seconds 5 > $O/bench.json 2> $O/bench.err &&
echo "level split" && timeout -k 10 300 python3 $R/profiles/level_split.py > $O/split.json 2> $O/split.err &&
lpmc() { local n=$1; shift; timeout -s KILL 300 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $O/$n -o pmc -- python3 $R/profiles/level_split.py --steps 2 > $O/$n.log 2>&1; }
echo "split pmc" && lpmc st TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum &&
lpmc sl TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE &&
lpmc sq SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES &&
echo "done"
