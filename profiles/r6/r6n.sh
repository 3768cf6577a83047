#!/bin/bash
# Round 6, call n: chain-kernel width on the lane-pair form: C4 at 8 / 10 /
# 12 waves (10 is the default for tables > 128 MiB), C5 at 10 / 12.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6n; mkdir -p $O
bash profiles/ab_opts.sh $O/c4b 2 w12:chain_waves=12 w14:chain_waves=14 w16:chain_waves=16 -- --config C4 || exit 1
bash profiles/ab_opts.sh $O/c5b 1 w12:chain_waves=12 w14:chain_waves=14 w16:chain_waves=16 -- --config C5 || exit 1
python3 - <<'PY'
import glob, json, os, collections
for d in ("c4", "c5", "c4b", "c5b"):
    acc = collections.defaultdict(list)
    for f in sorted(glob.glob("gpurun_out/r6n/%s/*.json" % d)):
        j = json.load(open(f))
        acc[os.path.basename(f).split(".")[0]].append("%.3f" % j["kernel_ms_per_launch"]["windows"])
    for v, xs in sorted(acc.items()):
        print(d, v, xs)
PY
