#!/bin/bash
# Collect rocprofv3 PMC counters for bench.py, one counter group per pass
# (FETCH_SIZE and WRITE_SIZE need their own passes on gfx950's TCC slots).
# usage (on the GPU box, from the repo root):
#   bash profiles/collect_pmc.sh gpurun_out/pmc [extra bench.py args]
OUT=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/$OUT"
cd /tmp && export TMPDIR=/tmp
run() {  # run NAME "COUNTERS" [bench args]
  local name=$1 ctr=$2; shift 2
  timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace --output-format csv \
      -d "$R/$OUT/$name" -o pmc -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu --host-steps 0 --latency-steps 0 "$@" \
      > "$R/$OUT/$name.json" 2> "$R/$OUT/$name.err"
}
run fetch "FETCH_SIZE" "$@" &&
run write "WRITE_SIZE" "$@" &&
run sq "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" "$@" &&
run sq2 "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT" "$@" &&
run tcc "TCC_HIT_sum TCC_MISS_sum" "$@"
