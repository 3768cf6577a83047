#!/bin/bash
# Memory-pipeline counters (TA / TCP / TCC / EA) for bench.py, one group per pass.
#   bash profiles/collect_mem.sh gpurun_out/mem [extra bench.py args]
OUT=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/$OUT"
cd /tmp && export TMPDIR=/tmp
run() {
  local name=$1 ctr=$2; shift 2
  timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace --output-format csv \
      -d "$R/$OUT/$name" -o pmc -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu "$@" \
      > "$R/$OUT/$name.json" 2> "$R/$OUT/$name.err"
}
run ea "TCC_EA0_RDREQ TCC_EA0_RDREQ_128B TCC_EA0_RDREQ_DRAM" "$@" &&
run ea2 "TCC_EA0_RDREQ_LEVEL TCC_EA0_RDREQ_DRAM_CREDIT_STALL" "$@" &&
run ta "TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TA_DATA_STALLED_BY_TC_CYCLES TA_TOTAL_WAVEFRONTS GRBM_GUI_ACTIVE" "$@" &&
run tcp "TCP_PENDING_STALL_CYCLES TCP_TCC_READ_REQ TCP_READ_TAGCONFLICT_STALL_CYCLES TCP_TA_TCP_STATE_READ" "$@" &&
run tcc "TCC_BUSY TCC_CYCLE TCC_TAG_STALL TCC_REQ" "$@"
