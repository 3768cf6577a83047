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
# the batch the PMC passes ran (bench.py's default for the config) keys pmc_windows.json
B=$(python3 -c "import json; print(json.load(open('$SRC/bench_traced.json'))['config']['frames_per_gpu_per_step'])")
python3 "$(dirname "$0")/pmc_summary.py" "$SRC/pmc" --batch "$B" --json "$(dirname "$0")/pmc_windows.json" > "$DST/pmc_summary.txt"
sed -i "s|\"source\": \".*\"|\"source\": \"$DST/pmc_*\"|" "$(dirname "$0")/pmc_windows.json"
