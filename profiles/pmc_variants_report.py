"""Per-variant window-kernel counters from profiles/pmc_variants.sh (per frame)."""
import collections
import csv
import glob
import os
import sys

d, frames = sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 8.0
res = collections.defaultdict(dict)
for f in glob.glob(os.path.join(d, "*", "pmc_counter_collection.csv")):
    v = os.path.basename(os.path.dirname(f)).split(".")[0]
    acc = collections.defaultdict(list)
    for row in csv.DictReader(open(f)):
        if any(k in row["Kernel_Name"] for k in ("cascade_kernel", "window_kernel", "chain_kernel")):
            acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, x in acc.items():
        res[v][k] = sum(x) / len(x) / frames
for v, cs in sorted(res.items()):
    hit = cs.get("TCC_HIT", 0) / max(cs.get("TCC_HIT", 0) + cs.get("TCC_MISS", 1), 1)
    print(v, "EA GB/frame %.2f" % (cs.get("TCC_EA0_RDREQ", 0) * 128 / 1e9), "L2 hit %.2f" % hit,
          " ".join("%s=%.3g" % (k, x) for k, x in sorted(cs.items())))
