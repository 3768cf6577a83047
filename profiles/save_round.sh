#!/bin/bash
# Copy one round_profile.sh result set from gpurun_out/ into profiles/ (tracked):
#   bash profiles/save_round.sh gpurun_out/r1c profiles/r1
SRC=$1; DST=$2
mkdir -p "$DST"
cp "$SRC/bench.json" "$SRC/bench_traced.json" "$DST/"
[ -f "$SRC/pytest.log" ] && cp "$SRC/pytest.log" "$DST/pytest_gpu.log"
cp "$SRC/trace/trace_kernel_stats.csv" "$DST/rocprof_kernel_stats.csv"
for p in "$SRC"/pmc/*/; do
  n=$(basename "$p"); mkdir -p "$DST/pmc_$n"
  cp "$p/pmc_counter_collection.csv" "$DST/pmc_$n/"
done
python3 "$(dirname "$0")/pmc_summary.py" "$SRC/pmc" --json "$(dirname "$0")/pmc_windows.json" > "$DST/pmc_summary.txt"
sed -i "s|\"source\": \".*\"|\"source\": \"$DST/pmc_*\"|" "$(dirname "$0")/pmc_windows.json"
