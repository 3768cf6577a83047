#!/bin/bash
# Round 6, call b: the lane-pair item form (SC_PAIR) in the chain kernel.
# Parity of the variant against the oracle, then interleaved A/B against the
# product build (C2, C4, one frame).  Variants: bash profiles/build_variants.sh
# base "" pair "-DSC_PAIR=1".
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6b; mkdir -p $O
SURFCASCADE_LIB=$R/surfcascade_amd/lib/variants/pair/libsurfcascade.so timeout -k 10 500 \
  python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_soak.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "grid_parity or chain or spec or waves or soak or subq or shard or ped or permissive" > $O/pytest_pair.log 2>&1 || { tail -30 $O/pytest_pair.log; exit 1; }
tail -2 $O/pytest_pair.log
bash profiles/ab.sh $O/c2 3 base pair || exit 1
bash profiles/ab.sh $O/c4 2 base pair -- --config C4 || exit 1
bash profiles/ab.sh $O/b1 3 base pair -- --batch 1 --steps 100 || exit 1
python3 - <<'PY'
import glob, json, os, collections
for d in ("c2", "c4", "b1"):
    acc = collections.defaultdict(list)
    for f in sorted(glob.glob("gpurun_out/r6b/%s/*.json" % d)):
        v = os.path.basename(f).split(".")[0]
        j = json.load(open(f))
        acc[v].append((j["ms_per_step"], j["kernel_ms_per_launch"]["windows"]))
    for v, xs in acc.items():
        print(d, v, "step", ["%.4f" % a for a, _ in xs], "chain", ["%.4f" % b for _, b in xs])
PY
