"""Summarise profiles/ab.sh output: per-variant window-kernel ms per frame (min/median)."""
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
    b = j["config"]["frames_per_gpu_per_step"]
    res.setdefault(v, []).append((j["kernel_ms_per_launch"]["windows"] / b, j["value"] / 1e9))
for v, xs in res.items():
    w = [x[0] for x in xs]
    print("%-8s windows ms/frame min %.4f med %.4f   Gwin/s max %.3f" % (v, min(w), statistics.median(w),
                                                                      max(x[1] for x in xs)))
