#!/bin/bash
# Round 6, call l: the fused column walk for interleaved cells as one wave per
# 32-column strip writing whole 32-B cells (both channel halves).  Parity of
# the walks on interleaved cells (product: table_layout 1 tests; pairall: the
# C2 bench form with every frame on lane pairs), then C2 base vs pairall, and
# C4 / C5 (interleaved by default) against round-5 numbers.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6l; mkdir -p $O
true || timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "fused or c4_bench_form or c5_bench_form" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
SC_TEST_ANY_ITEM_FORM=1 SURFCASCADE_LIB=$R/surfcascade_amd/lib/variants/pairall/libsurfcascade.so timeout -k 10 300 \
  python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "c2_bench_form_exact" > $O/pytest_pairall.log 2>&1 || { tail -30 $O/pytest_pairall.log; exit 1; }
tail -1 $O/pytest_pairall.log
bash profiles/ab.sh $O/c2 2 base pairall || exit 1
bash profiles/ab.sh $O/c4 1 base -- --config C4 || exit 1
bash profiles/ab.sh $O/c5 1 base -- --config C5 || exit 1
python3 - <<'PY'
import glob, json, os
for d in ("c2", "c4", "c5"):
    for f in sorted(glob.glob("gpurun_out/r6l/%s/*.json" % d)):
        j = json.load(open(f))
        print(d, os.path.basename(f), "%.4f ms/step chain %.4f %.3f G" % (j["ms_per_step"], j["kernel_ms_per_launch"]["windows"], j["value"] / 1e9))
PY
