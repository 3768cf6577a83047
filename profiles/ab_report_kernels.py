"""Summarise profiles/ab.sh output per variant: every kernel's ms per launch
(min / median over the interleaved runs) and the bench value."""
import glob
import json
import os
import statistics
import sys

d = sys.argv[1]
res = {}
for f in sorted(glob.glob(os.path.join(d, "*.json"))):
    v = os.path.basename(f).split(".")[0]
    j = json.load(open(f))
    res.setdefault(v, []).append(j)
for v, js in res.items():
    ks = js[0]["kernel_ms_per_launch"].keys()
    parts = []
    for k in ks:
        xs = [j["kernel_ms_per_launch"][k] for j in js]
        parts.append("%s %.4f/%.4f" % (k, min(xs), statistics.median(xs)))
    print("%-8s %s  Gwin/s max %.3f" % (v, "  ".join(parts), max(j["value"] for j in js) / 1e9))
