#!/bin/bash
# Round 3, call 7: PMC passes for C2, C4, C5 with the product build
# (profiles/collect_pmc_cfg.sh), then pmc_windows.json keyed per config.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r3g7
mkdir -p $R/$O
cd $R
for c in C2 C4 C5; do
  echo "pmc $c" && bash profiles/collect_pmc_cfg.sh $O/$c --config $c || exit 1
done
echo ok
