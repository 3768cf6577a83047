"""Summarise profiles/ab.sh output per variant: every kernel's ms per launch
(min / median over the interleaved runs) and the bench value.  Reads the raw
NAME.R.json run files and / or DIR/runs.json (profiles/fold_runs.py)."""
import glob
import json
import os
import re
import statistics
import sys

d = sys.argv[1]
res = {}
runs = {}
if os.path.exists(os.path.join(d, "runs.json")):
    runs.update(json.load(open(os.path.join(d, "runs.json"))))
for f in sorted(glob.glob(os.path.join(d, "*.json"))):
    m = re.match(r"^(.+)\.(\d+)\.json$", os.path.basename(f))
    if m:
        runs[m.group(1) + "." + m.group(2)] = json.load(open(f))
for key in sorted(runs):
    j = runs[key]
    if isinstance(j, dict) and "kernel_ms_per_launch" in j:
        res.setdefault(key.split(".")[0], []).append(j)
for v, js in res.items():
    ks = js[0]["kernel_ms_per_launch"].keys()
    parts = []
    for k in ks:
        xs = [j["kernel_ms_per_launch"][k] for j in js]
        parts.append("%s %.4f/%.4f" % (k, min(xs), statistics.median(xs)))
    print("%-8s %s  Gwin/s max %.3f" % (v, "  ".join(parts), max(j["value"] for j in js) / 1e9))
