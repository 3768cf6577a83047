#!/bin/bash
# Round 6, call u: batch launch knobs re-checked at the final build: frames
# integrated before the chain kernel (C2 / C5: 1 / 3 vs 2; C4: 2 vs 1) and
# C2 with 4 segments per row.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6u; mkdir -p $O
bash profiles/ab_opts.sh $O/c2 3 d: pre1:integral_pre=1 pre3:integral_pre=3 sg4:chain_segs=4 || exit 1
bash profiles/ab_opts.sh $O/c5 2 d: pre1:integral_pre=1 pre3:integral_pre=3 -- --config C5 || exit 1
bash profiles/ab_opts.sh $O/c4 2 d: pre2:integral_pre=2 -- --config C4 || exit 1
python3 - <<'PY'
import glob, json, os, collections
for d in ("c2", "c5", "c4"):
    acc = collections.defaultdict(list)
    for f in sorted(glob.glob("gpurun_out/r6u/%s/*.json" % d)):
        j = json.load(open(f))
        acc[os.path.basename(f).split(".")[0]].append("%.3f/%.3f" % (j["ms_per_step"], j["kernel_ms_per_launch"]["windows"]))
    for v, xs in sorted(acc.items()):
        print(d, v, xs)
PY
