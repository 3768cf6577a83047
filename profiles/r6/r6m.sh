#!/bin/bash
# Round 6, call m: one frame per call, the speculative rounds aimed at the
# waiting task of the later segment first (SC_SPEC_PRIO; segment 3 waits
# longest, profiles/r6/k), with 1 and 2 rounds per task.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6m; mkdir -p $O
SURFCASCADE_LIB=$R/surfcascade_amd/lib/variants/prio/libsurfcascade.so timeout -k 10 300 \
  python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "speculat or one_frame" > $O/pytest_prio.log 2>&1 || { tail -30 $O/pytest_prio.log; exit 1; }
tail -1 $O/pytest_prio.log
bash profiles/ab.sh $O/b1 3 base prio -- --batch 1 --steps 200 || exit 1
bash profiles/ab.sh $O/b1s2 2 base prio -- --batch 1 --steps 200 --opt chain_spec=2 || exit 1
python3 - <<'PY'
import glob, json, os, collections
for d in ("b1", "b1s2"):
    acc = collections.defaultdict(list)
    for f in sorted(glob.glob("gpurun_out/r6m/%s/*.json" % d)):
        j = json.load(open(f))
        acc[os.path.basename(f).split(".")[0]].append("%.4f/%.4f" % (j["ms_per_step"], j["kernel_ms_per_launch"]["windows"]))
    for v, xs in sorted(acc.items()):
        print(d, v, xs)
PY
