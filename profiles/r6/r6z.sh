#!/bin/bash
# Round 6, call z: more soak at the final build (large single frames among
# the cases): seeds 33000 and 36000, 200 cases each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=$R/gpurun_out/r6z; mkdir -p $O
for sd in 33000 36000; do
  timeout -k 10 560 python3 -u tests/soak_parity.py --cases 200 --seed $sd --out $O/soak_$sd.json > $O/soak_$sd.log 2>&1; rc=$?
  tail -2 $O/soak_$sd.log | cut -c1-300
  [ $rc -eq 0 ] || exit 1
done
