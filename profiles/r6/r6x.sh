#!/bin/bash
# Round 6, call x: row blocks of the batch task order re-checked on the
# lane-pair form at 12 waves (C4, C5): 16 / 48 vs 32 grid rows.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6x; mkdir -p $O
bash profiles/ab_opts.sh $O/c4 2 d: rb16:row_block=16 rb48:row_block=48 -- --config C4 || exit 1
bash profiles/ab_opts.sh $O/c5 2 d: rb16:row_block=16 rb48:row_block=48 -- --config C5 || exit 1
python3 - <<'PY'
import glob, json, os, collections
for d in ("c4", "c5"):
    acc = collections.defaultdict(list)
    for f in sorted(glob.glob("gpurun_out/r6x/%s/*.json" % d)):
        j = json.load(open(f))
        acc[os.path.basename(f).split(".")[0]].append("%.3f/%.3f" % (j["ms_per_step"], j["kernel_ms_per_launch"]["windows"]))
    for v, xs in sorted(acc.items()):
        print(d, v, xs)
PY
