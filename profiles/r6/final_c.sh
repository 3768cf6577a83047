#!/bin/bash
# Round 6 evidence, part C: the C2 / C4 / C5 bench lines again after
# save_final.sh re-keyed profiles/pmc_windows.json on part B's passes (same
# build), so every committed line carries its PMC-derived roofline fields.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=gpurun_out/r6final; mkdir -p $R/$O; cd $R
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 400 python3 bench.py --config C4 > $O/bench_C4.json 2> $O/bench_C4.err || exit 1
timeout -k 10 400 python3 bench.py --config C5 > $O/bench_C5.json 2> $O/bench_C5.err || exit 1
python3 - <<'PY'
import json
for f in ("bench", "bench_C4", "bench_C5"):
    d = json.load(open("gpurun_out/r6final/%s.json" % f))
    r = d["roofline"]
    print(f, "%.3f G" % (d["value"] / 1e9), "frac %.4f" % r["frac"], "traffic", r.get("traffic"), "fabric", r.get("fabric_frac"),
          "td", r.get("td_busy_frac"), "l2", r.get("l2_hit"), "stale", r.get("pmc_stale"), d["config"].get("item_form"))
PY
