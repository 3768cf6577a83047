#!/bin/bash
# Round 5 soak: the parity soak (tests/soak_parity.py), then the chain kernel's per-launch
# durations over 300 C2 steps and 2000 one-frame steps (rocprofv3 kernel
# trace): tail latency of the persistent kernel on the kept build.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=$R/gpurun_out/soak; mkdir -p $O
timeout -k 10 300 python3 -u tests/soak_parity.py --cases 8 --seed 1 > $O/soak_smoke.log 2>&1 || { tail -20 $O/soak_smoke.log; exit 1; }
tail -1 $O/soak_smoke.log | cut -c1-300
timeout -k 10 1000 python3 -u tests/soak_parity.py --cases 300 --seed 9000 --out $O/soak.json > $O/soak.log 2>&1; rc=$?
tail -3 $O/soak.log | cut -c1-400
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
( cd /tmp && export TMPDIR=/tmp &&
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/c2 -o trace -- python3 $R/bench.py --no-cpu \
    --latency-steps 0 --host-steps 0 --steps 300 --warmup 3 > $O/c2.json 2> $O/c2.err ) || exit 1
( cd /tmp && export TMPDIR=/tmp &&
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/b1 -o trace -- python3 $R/bench.py --no-cpu \
    --latency-steps 0 --host-steps 0 --batch 1 --steps 2000 --warmup 3 > $O/b1.json 2> $O/b1.err ) || exit 1
for t in c2 b1; do
  python3 - $O/$t/trace_kernel_trace.csv $t <<'PY'
import csv, sys
import numpy as np
ch = [r for r in csv.DictReader(open(sys.argv[1])) if 'chain_kernel' in r['Kernel_Name']]
d = np.array([(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6 for r in ch])
print(sys.argv[2], "launches", len(d), "median %.4f p99 %.4f p99.9 %.4f max %.4f ms" % (
    np.median(d), np.percentile(d, 99), np.percentile(d, 99.9), d.max()), "max at launch", int(d.argmax()))
PY
done
echo soak done
