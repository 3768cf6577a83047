#!/bin/bash
# Round 5: the kept build (vector sc1 polls) under the same rocprofv3 C2
# command twice (per-launch durations: does a >15 ms launch appear without
# the scalar polls?), and the one-frame latency legs on this build.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r5recheck; mkdir -p $O
bash profiles/run.sh r5recheck "rocprof trace1" "rocprof trace2" || exit 1
for t in trace1 trace2; do
  python3 - $O/$t/trace_kernel_trace.csv <<'PY'
import csv, sys
ch = [r for r in csv.DictReader(open(sys.argv[1])) if 'chain_kernel' in r['Kernel_Name']]
print(" ".join("%.3f" % ((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6) for r in ch))
PY
done
timeout -k 10 240 python3 profiles/r5/latency_legs.py > $O/legs.json 2> $O/legs.err || exit 1
cat $O/legs.json
