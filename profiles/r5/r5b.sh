#!/bin/bash
# Round 5, second GPU call: the drained-tail rounds and the per-launch
# sub-queue count on the one-frame path (interleaved option A/B), the same
# in batches (C2), rowcarry4's load depth (variants rc2 / rc4 vs 8), the
# pipelined LDS-DMA item loop (itembench V16) with its counters, and the
# single-frame grid split's balance on one GPU.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R
PYTEST_K="tail_rounds_match or four_subqueues or speculative or integral" bash profiles/run.sh r5b "pytest" \
  "abopt b1 3 base: t1:chain_tail=1 q2:chain_subq=2 q8:chain_subq=8 q1:chain_subq=1 -- --batch 1 --steps 50" \
  "abopt c2 2 base: t2:chain_tail=2" \
  "ab rcb1 3 rc2 rc4 -- --batch 1 --steps 50" \
  "ab rcc2 2 rc2 -- --steps 10" \
  "itembench --variants 0:12,0:16,0:6,0:4,16:6,16:4,15:12 --reps 7 --out gpurun_out/r5b/ib.json" || exit 1
V=0:12,0:6,16:6 IBPMC_OUT=r5b/ibpmc timeout -k 10 600 bash profiles/itembench/ib_pmc.sh || exit 1
timeout -k 10 300 python3 profiles/shard_balance.py --config C2 > gpurun_out/r5b/shard_c2.txt 2>&1 || exit 1
timeout -k 10 400 python3 profiles/shard_balance.py --config C4 --steps 10 > gpurun_out/r5b/shard_c4.txt 2>&1 || exit 1
echo done
