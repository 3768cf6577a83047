#!/bin/bash
# Round 3, call 21: C1 (CPU-only line), C4 and C5 bench lines, then the PMC
# passes of C2 on the fused-integral build.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r3g21
mkdir -p $O
cd $R
for c in C1 C4 C5; do
  timeout -k 10 400 python3 bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 1; }
  cut -c1-300 $O/bench_$c.json
done
bash profiles/collect_pmc_cfg.sh gpurun_out/r3g21/C2 --config C2 && echo pmc ok
