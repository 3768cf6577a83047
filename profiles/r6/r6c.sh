#!/bin/bash
# Round 6, call c: counters of the lane-pair chain kernel against the product
# build (C2, C4): L2 hits / misses, L1->L2 requests, L1 accesses, VALU and
# vector-memory instructions (profiles/pmc_variants.sh), and the product build
# with interleaved cells but the one-lane item form (table_layout=1).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6c; mkdir -p $O
bash profiles/pmc_variants.sh $O/c2 base pair || exit 1
bash profiles/pmc_variants.sh $O/c4 base pair -- --config C4 || exit 1
bash profiles/ab.sh $O/inter 2 base -- --opt table_layout=1 || exit 1
bash profiles/ab.sh $O/inter4 1 base -- --opt table_layout=1 --config C4 || exit 1
echo done
