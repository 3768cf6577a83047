#!/bin/bash
# Round 4: beyond-L2 row-gather ceilings (profiles/calib k_rows_*), and the
# C4 chain kernel split by level group (levels 0-23 = C2's window sizes on a
# 4K table; 24-31 the widest) beside C2, for the per-item cost analysis.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=gpurun_out/r4c4; mkdir -p $R/$O; cd $R
timeout -k 10 120 profiles/calib/fetch_calib > $O/calib.txt 2>&1 || exit 1
grep k_rows $O/calib.txt
B="timeout -k 10 200 python3 bench.py --steps 6 --warmup 2 --no-cpu --latency-steps 0 --host-steps 0"
$B --config C2 > $O/c2.json 2> $O/c2.err || exit 1
$B --config C4 > $O/c4.json 2> $O/c4.err || exit 1
$B --config C4 --opt level_hi=24 > $O/c4_lo.json 2> $O/c4_lo.err || exit 1
$B --config C4 --opt level_lo=24 > $O/c4_hi.json 2> $O/c4_hi.err || exit 1
$B --config C2 --opt level_hi=13 > $O/c2_lo.json 2> $O/c2_lo.err || exit 1
$B --config C2 --opt level_lo=13 > $O/c2_hi.json 2> $O/c2_hi.err || exit 1
for f in c2 c4 c4_lo c4_hi c2_lo c2_hi; do python3 -c "import json;d=json.load(open('$O/$f.json'));print('$f', d['kernel_ms_per_launch']['windows'], d['visited_windows_last_step'])"; done
