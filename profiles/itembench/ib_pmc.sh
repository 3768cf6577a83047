#!/bin/bash
# PMC passes over the item-loop variants (TA / TD / TCP / SQ / TCC), one
# rocprofv3 run per counter group; run on the GPU box from the repo root
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${IBPMC_OUT:-ibpmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
V=${V:-0:12,4:16,2:12}
run() { local n=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $OUT/$n -o pmc -- \
    python3 $R/profiles/itembench/run.py --variants $V --reps 2 > $OUT/$n.log 2>&1; }
run p1 TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_UTCL1_TRANSLATION_MISS_sum GRBM_GUI_ACTIVE &&
[ -n "$ONLY1" ] || run p2 TA_DATA_STALLED_BY_TC_CYCLES_sum TA_FLAT_READ_WAVEFRONTS_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TD_LOAD_WAVEFRONT_sum TD_COALESCABLE_WAVEFRONT_sum &&
run p3 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY &&
run p4 TCC_HIT_sum TCC_MISS_sum &&
run p5 SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_WAVES GRBM_GUI_ACTIVE
