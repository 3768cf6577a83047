#!/bin/bash
# Memory-pipeline counters (TA / TD / TCP / SQ) for bench.py's kernels, one
# rocprofv3 pass per counter group.  usage (GPU box, repo root):
#   bash profiles/collect_pmc_ta.sh gpurun_out/tapmc [extra bench.py args]
OUT=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/$OUT"
cd /tmp && export TMPDIR=/tmp
run() {
  local name=$1 ctr=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$R/$OUT/$name" -o pmc -- \
      python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu --host-steps 0 --latency-steps 0 "$@" \
      > "$R/$OUT/$name.json" 2> "$R/$OUT/$name.err"
}
run ta1 "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum GRBM_GUI_ACTIVE" "$@" &&
run sq1 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" "$@" &&
run sq2 "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INSTS_BRANCH" "$@"
