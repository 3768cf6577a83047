#!/bin/bash
# Copy gpurun_out/r6final (final_a.sh + final_b.sh) into profiles/r6/final (tracked) and re-key
# profiles/pmc_windows.json (C2 / C4 / C5) on its PMC passes: each entry
# carries the build id of the library the passes profiled.
set -e
S=gpurun_out/r6final; D=profiles/r6/final
mkdir -p $D
cp $S/bench.json $S/bench_C1.json $S/bench_C4.json $S/bench_C5.json $D/
cp $S/pytest.log $S/smoke.log $S/legs.json $D/
cp $S/trace/trace_kernel_stats.csv $D/rocprof_kernel_stats_c2.csv
cp $S/trace_b1/trace_kernel_stats.csv $D/rocprof_kernel_stats_b1.csv
for c in C2 C4 C5; do
  mkdir -p $D/pmc/$c
  for p in $S/pmc/$c/*/; do n=$(basename $p); cp $p/pmc_counter_collection.csv $D/pmc/$c/$n.csv; done
  cp $S/pmc/$c/*.json $D/pmc/$c/
done
python3 profiles/pmc_summary.py $S/pmc/C2 --config C2 --batch 32 --json profiles/pmc_windows.json > $D/pmc_summary_C2.txt
python3 profiles/pmc_summary.py $S/pmc/C4 --config C4 --batch 8 --width 3840 --height 2160 --levels 32 \
  --json profiles/pmc_windows.json > $D/pmc_summary_C4.txt
python3 profiles/pmc_summary.py $S/pmc/C5 --config C5 --batch 32 --levels 23 --json profiles/pmc_windows.json \
  > $D/pmc_summary_C5.txt
python3 - <<'PY'
import json
p = "profiles/pmc_windows.json"
d = json.load(open(p))
for c in ("C2", "C4", "C5"):
    d["configs"][c]["source"] = "profiles/r6/final/pmc/" + c
json.dump(d, open(p, "w"), indent=1)
PY
echo saved
