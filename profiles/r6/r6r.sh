#!/bin/bash
# Round 6, call r: one frame per call at one task per wave: dequeue
# sub-queues (8 default vs 4), bottom-up row blocks (4 default vs 2 / 8),
# 10 waves.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6r; mkdir -p $O
bash profiles/ab_opts.sh $O/b1q 3 q4:chain_subq=4 q1:chain_subq=1 q2:chain_subq=2 q3:chain_subq=3 -- --batch 1 --steps 200 || exit 1
python3 - <<'PY'
import glob, json, os, collections
acc = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/r6r/b1q/*.json")):
    j = json.load(open(f))
    acc[os.path.basename(f).split(".")[0]].append("%.4f/%.4f" % (j["ms_per_step"], j["kernel_ms_per_launch"]["windows"]))
for v, xs in sorted(acc.items()):
    print("b1", v, xs)
PY
