#!/bin/bash
# rocprofv3 PMC passes over bench.py for one config (one counter group per
# pass; gfx950 slot limits: 8 SQ, 4 TCC (FETCH_SIZE takes 3, WRITE_SIZE 2),
# 4 TCP, 2 TA, 2 TD, 2 GRBM).  Run on the GPU box from the repo root:
#   bash profiles/collect_pmc_cfg.sh OUTDIR [bench.py args, e.g. --config C4]
OUT=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/$OUT"
cd /tmp && export TMPDIR=/tmp
run() {  # run NAME COUNTERS...
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$R/$OUT/$name" -o pmc -- \
      python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu --host-steps 0 --latency-steps 0 $BENCH_ARGS \
      > "$R/$OUT/$name.json" 2> "$R/$OUT/$name.err"
}
BENCH_ARGS="$*"
run fetch FETCH_SIZE &&
run write WRITE_SIZE &&
run tcc TCC_HIT_sum TCC_MISS_sum &&
run sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY &&
run sq2 SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM &&
run tcp TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE &&
run ta TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum
