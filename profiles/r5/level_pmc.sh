#!/bin/bash
# PMC passes of the chain kernel restricted to one level range (SC_OPT_LEVEL_LO/_HI
# via profiles/level_split.py), one rocprofv3 run per counter group (gfx950 slot
# limits: 8 SQ, 4 TCC, 4 TCP, 2 TA, 2 TD, 2 GRBM).  Run on the GPU box from the
# repo root:  bash profiles/r5/level_pmc.sh OUTDIR LO:HI [level_split.py args]
# Summary: python3 profiles/r5/level_pmc_report.py OUTDIR ...
OUT=$1; RG=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
D=$R/$OUT/${RG/:/_}
mkdir -p "$D"
cd /tmp && export TMPDIR=/tmp
run() {  # run NAME COUNTERS...
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$D/$name" -o pmc -- \
      python3 "$R/profiles/level_split.py" --ranges "$RG" --steps 2 $SPLIT_ARGS > "$D/$name.json" 2> "$D/$name.err"
}
SPLIT_ARGS="$*"
run tcc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE &&
run sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_SALU &&
run td TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE
