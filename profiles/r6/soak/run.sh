#!/bin/bash
# Round 6 soak at the final build: 600 random parity cases through the C ABI
# against the oracle (tests/soak_parity.py; the cell layout -- split or
# interleaved, i.e. the one-lane or the lane-pair item form -- is one of the
# drawn options), and the chain kernel's per-launch durations over 100 C4
# steps (the lane-pair form at 12 waves).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=$R/gpurun_out/soak6; mkdir -p $O
for sd in 21000 24000; do
  timeout -k 10 500 python3 -u tests/soak_parity.py --cases 300 --seed $sd --out $O/soak_$sd.json > $O/soak_$sd.log 2>&1; rc=$?
  tail -2 $O/soak_$sd.log | cut -c1-300
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
done
( cd /tmp && export TMPDIR=/tmp &&
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/c4 -o trace -- python3 $R/bench.py --no-cpu \
    --latency-steps 0 --host-steps 0 --config C4 --steps 100 --warmup 3 > $O/c4.json 2> $O/c4.err ) || exit 1
python3 - $O/c4/trace_kernel_trace.csv <<'PY'
import csv, sys, statistics
d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(sys.argv[1]))
     if "chain_kernel" in r["Kernel_Name"]]
d = [x / 1e6 for x in d]
s = sorted(d[3:])
print("C4 chain launches %d median %.3f p99 %.3f max %.3f first %.3f" % (len(d), statistics.median(s), s[int(0.99 * (len(s) - 1))], max(s), d[0]))
PY
