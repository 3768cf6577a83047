#!/bin/bash
# PMC of the chain kernel with and without the packed (u24) table, fusion off
R=${GRAFT_REPO_ROOT:-$(pwd)}
for u in 1 2; do
  BENCH="--opt integral_fuse=1 --opt table_u24=$u"
  O=gpurun_out/u24pmc/u$u
  mkdir -p "$R/$O"
  ( cd /tmp && export TMPDIR=/tmp &&
    for pass in "tcc:TCC_HIT_sum TCC_MISS_sum" "tcp:TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE" "ta:TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum" "sq:SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU"; do
      name=${pass%%:*}; ctr=${pass#*:}
      timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$R/$O/$name" -o pmc -- \
        python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu --host-steps 0 --latency-steps 0 $BENCH \
        > "$R/$O/$name.json" 2> "$R/$O/$name.err" || exit 1
    done ) || exit 1
done
