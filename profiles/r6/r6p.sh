#!/bin/bash
# Round 6, call p: one frame per call with one task per wave (chain_slots 1)
# against the default 2, and with 2 / 4 speculative rounds per task.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6p; mkdir -p $O
bash profiles/ab_opts.sh $O/b1 3 s2: s1:chain_slots=1 s1sp2:chain_slots=1,chain_spec=2 s1sp4:chain_slots=1,chain_spec=4 -- --batch 1 --steps 200 || exit 1
bash profiles/ab_opts.sh $O/c2 1 s2: s1:chain_slots=1 || exit 1
python3 - <<'PY'
import glob, json, os, collections
for d in ("b1", "c2"):
    acc = collections.defaultdict(list)
    for f in sorted(glob.glob("gpurun_out/r6p/%s/*.json" % d)):
        j = json.load(open(f))
        acc[os.path.basename(f).split(".")[0]].append("%.4f/%.4f" % (j["ms_per_step"], j["kernel_ms_per_launch"]["windows"]))
    for v, xs in sorted(acc.items()):
        print(d, v, xs)
PY
