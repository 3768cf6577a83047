#!/bin/bash
# Round 6 evidence at HEAD, part B: the PMC passes of C2 / C4 / C5
# (profiles/collect_pmc_cfg.sh; the pmc_windows.json sources).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=gpurun_out/r6final; mkdir -p $R/$O; cd $R
for c in C2 C4 C5; do bash profiles/collect_pmc_cfg.sh $O/pmc/$c --config $c || exit 1; echo "pmc $c done"; done
echo final_b done
