#!/bin/bash
# Round 6, call f: where the lane-pair form pays.  C2 with it at 12 waves
# (the 16-wave kernel runs the one-lane form on split cells), one frame per
# call with and without it.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6f; mkdir -p $O
bash profiles/ab.sh $O/c2w12 2 pairall -- --opt chain_waves=12 || exit 1
bash profiles/ab.sh $O/c2 2 base pairall || exit 1
bash profiles/ab.sh $O/b1 3 base pairall -- --batch 1 --steps 200 || exit 1
python3 - <<'PY'
import glob, json, os, collections
for d in ("c2w12", "c2", "b1"):
    acc = collections.defaultdict(list)
    for f in sorted(glob.glob("gpurun_out/r6f/%s/*.json" % d)):
        v = os.path.basename(f).split(".")[0]
        j = json.load(open(f))
        acc[v].append((j["ms_per_step"], j["kernel_ms_per_launch"]["windows"]))
    for v, xs in sorted(acc.items()):
        print(d, v, "step", ["%.4f" % a for a, _ in xs], "chain", ["%.4f" % b for _, b in xs])
PY
