#!/bin/bash
# Round 6, call w: one frame per call at one task per wave: task order
# (row_order 1 y-major, 2 top-down blocks vs 3 bottom-up blocks) and 2
# segments per row.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6w; mkdir -p $O
bash profiles/ab_opts.sh $O/b1 3 d: ro1:row_order=1 ro2:row_order=2 sg2:chain_segs=2 -- --batch 1 --steps 200 || exit 1
python3 - <<'PY'
import glob, json, os, collections
acc = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/r6w/b1/*.json")):
    j = json.load(open(f))
    acc[os.path.basename(f).split(".")[0]].append("%.4f/%.4f" % (j["ms_per_step"], j["kernel_ms_per_launch"]["windows"]))
for v, xs in sorted(acc.items()):
    print("b1", v, xs)
PY
