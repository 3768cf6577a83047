#!/bin/bash
# Round 6, call h: does the interleaved cell layout cost C2 in its fused
# column walks (16-B stores at 32-B stride from two waves per column strip)?
# C2 without fusion (integral_fuse 1: the column pass by its own kernels),
# split cells (base) vs interleaved + lane pairs (pairall).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6h; mkdir -p $O
bash profiles/ab.sh $O/nofuse 2 base pairall -- --opt integral_fuse=1 || exit 1
bash profiles/ab.sh $O/fuse 1 base pairall || exit 1
python3 - <<'PY'
import glob, json, os
for d in ("nofuse", "fuse"):
    for f in sorted(glob.glob("gpurun_out/r6h/%s/*.json" % d)):
        j = json.load(open(f))
        k = j["kernel_ms_per_launch"]
        print(d, os.path.basename(f), "%.4f ms/step" % j["ms_per_step"], {a: round(b, 4) for a, b in k.items()})
PY
