#!/bin/bash
# Round 6, call g: the product build with the lane-pair form chosen per
# geometry (C4, C5: interleaved cells, lane pairs; C2, one frame: split cells):
# the GPU suite, then old (round 5, SC_PAIR=0) vs base on C2 / C4 / C5 / one frame.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6g; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash profiles/ab.sh $O/c2 1 old base || exit 1
bash profiles/ab.sh $O/c4 1 old base -- --config C4 || exit 1
bash profiles/ab.sh $O/c5 1 old base -- --config C5 || exit 1
bash profiles/ab.sh $O/b1 1 old base -- --batch 1 --steps 200 || exit 1
python3 - <<'PY'
import glob, json, os
for d in ("c2", "c4", "c5", "b1"):
    for f in sorted(glob.glob("gpurun_out/r6g/%s/*.json" % d)):
        j = json.load(open(f))
        print(d, os.path.basename(f), "%.4f ms/step %.4f chain %.3f G" % (j["ms_per_step"], j["kernel_ms_per_launch"]["windows"], j["value"] / 1e9))
PY
