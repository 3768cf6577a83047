#!/bin/bash
# Round 6, call j: the single-frame split with 8 / 2 segments per row
# (SC_OPT_CHAIN_SEGS; one-frame launches default to 4), and the counters of
# the wide-level cap on C4 (cap 6 vs the default) for its negative.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6j; mkdir -p $O
for sg in 8 2; do
  timeout -k 10 200 python3 profiles/shard_balance.py --config C2 --opt chain_segs=$sg > $O/shard_c2_s$sg.txt 2> $O/shard_c2_s$sg.err || exit 1
  tail -1 $O/shard_c2_s$sg.txt > $O/shard_c2_s$sg.json
done
bash profiles/pmc_variants.sh $O/pmc4 base cap6 -- --config C4 || exit 1
python3 - <<'PY'
import json
for sg in (8, 2):
    d = json.load(open("gpurun_out/r6j/shard_c2_s%d.json" % sg))
    for w, v in d["worlds"].items():
        r = v["ranks"]
        print("c2 segs", sg, w, "chain max %.4f" % max(x["chain_ms"] for x in r), "eff %.3f" % v["implied_strong_efficiency"])
PY
python3 profiles/pmc_variants_report.py $O/pmc4
