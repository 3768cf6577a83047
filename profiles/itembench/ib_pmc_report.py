"""Summarise profiles/itembench/ib_pmc.sh output: per item-loop kernel, the
mean of each counter over its dispatches (one column per kernel)."""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(d, "*", "pmc_counter_collection.csv")):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"]
        if "k_" not in k:
            continue
        name = k[k.index("k_"):].split("(")[0].split("E")[0]
        acc[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
ks = sorted(acc)
ctr = sorted({c for k in ks for c in acc[k]})
print("%-40s" % "" + "".join("%16s" % k for k in ks))
for c in ctr:
    print("%-40s" % c + "".join("%16.4g" % (sum(acc[k][c]) / len(acc[k][c]) if acc[k][c] else 0) for k in ks))
