#!/bin/bash
# Round 6, call q: one frame per call with one task per wave (now the
# default): the chain kernel's width (12 / 14 / 16 waves; speculation runs in
# the 12-wave kernel only) and segments per row (4 / 8); parity of one-frame
# launches at the new default.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6q; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "one_frame or speculat or shard or subq or grid_parity_1080p or reference_level or chain_row_orders or waves" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash profiles/ab_opts.sh $O/b1 3 d: w14:chain_waves=14 w16:chain_waves=16 sg8:chain_segs=8 -- --batch 1 --steps 200 || exit 1
python3 - <<'PY'
import glob, json, os, collections
acc = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/r6q/b1/*.json")):
    j = json.load(open(f))
    acc[os.path.basename(f).split(".")[0]].append("%.4f/%.4f" % (j["ms_per_step"], j["kernel_ms_per_launch"]["windows"]))
for v, xs in sorted(acc.items()):
    print("b1", v, xs)
PY
