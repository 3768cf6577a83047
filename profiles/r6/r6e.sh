#!/bin/bash
# Round 6, call e: with the lane-pair form now the default for tables above
# 128 MiB (base; old = the round-5 one-lane form everywhere), a cap on the task
# slots of a CU that hold a wide-level row (SC_WIDECAP; the wide levels' rows
# dealt from a list of their own): parity of one variant, then C4 (wide = l >=
# 690, levels 24-31) with caps 6 / 10 / 14 of the 10-wave kernel's 20 slots
# and C2 (wide = l >= 241, levels 13-23) with caps 8 / 16 of the 16-wave
# kernel's 32; C2 / C5 with the pair form for every frame (pairall).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6e; mkdir -p $O
SURFCASCADE_LIB=$R/surfcascade_amd/lib/variants/cap6/libsurfcascade.so timeout -k 10 400 \
  python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "bench_form_exact or grid_parity_1080p or c4_grid_parity or kernel_paths or reference_level" > $O/pytest_cap6.log 2>&1 || { tail -30 $O/pytest_cap6.log; exit 1; }
tail -1 $O/pytest_cap6.log
SURFCASCADE_LIB=$R/surfcascade_amd/lib/variants/c2cap8/libsurfcascade.so timeout -k 10 300 \
  python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "c2_bench_form_exact or c5_bench_form_exact" > $O/pytest_c2cap8.log 2>&1 || { tail -30 $O/pytest_c2cap8.log; exit 1; }
tail -1 $O/pytest_c2cap8.log
bash profiles/ab.sh $O/c4 2 old base cap6 cap10 cap14 -- --config C4 || exit 1
bash profiles/ab.sh $O/c2 2 old base pairall c2cap8 c2cap16 || exit 1
bash profiles/ab.sh $O/c5 2 base pairall -- --config C5 || exit 1
python3 - <<'PY'
import glob, json, os, collections
for d in ("c4", "c2", "c5"):
    acc = collections.defaultdict(list)
    for f in sorted(glob.glob("gpurun_out/r6e/%s/*.json" % d)):
        v = os.path.basename(f).split(".")[0]
        j = json.load(open(f))
        acc[v].append(j["kernel_ms_per_launch"]["windows"])
    for v, xs in sorted(acc.items()):
        print(d, v, "chain", ["%.3f" % b for b in xs])
PY
