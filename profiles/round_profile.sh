#!/bin/bash
# One round's measurement set (run on the GPU box from the repo root):
#   bench.py default line, rocprofv3 kernel-trace stats of the same command,
#   PMC passes for the window kernel's HBM traffic.
#   bash profiles/round_profile.sh gpurun_out/rN
OUT=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/$OUT"
timeout -k 10 400 python3 "$R/bench.py" > "$R/$OUT/bench.json" 2> "$R/$OUT/bench.err" &&
( cd /tmp && export TMPDIR=/tmp &&
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/trace" -o trace \
      -- python3 "$R/bench.py" --no-cpu --latency-steps 0 --host-steps 0 > "$R/$OUT/bench_traced.json" 2> "$R/$OUT/trace.err" ) &&
bash "$R/profiles/collect_pmc.sh" "$OUT/pmc"
