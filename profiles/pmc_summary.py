"""Summarise rocprofv3 --pmc passes (profiles/collect_pmc.sh) per kernel.

HBM bytes per launch follow MI355X_MICROARCH.md's HBM section: FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide
coalesced streaming read, so it is doubled (uncalibrated for other access
shapes -- see DESIGN.md).
usage: python profiles/pmc_summary.py gpurun_out/pmc1 [--json out.json --batch 16 ...]
"""
import argparse
import collections
import csv
import glob
import json
import os

KERNELS = {"window_kernel": "windows", "cascade_kernel": "windows", "chain_kernel": "windows",
           "walk_kernel": "walk",
           "rowscan_kernel": "rowscan", "colscan_kernel": "colscan",
           "rowcarry_kernel": "rowscan", "colstrip_kernel": "colscan"}


def load(d):
    """Per kernel and counter, the mean over the batch's launches.  A pass may
    also hold launches of another shape (a batch-1 leg, a chunk tail): only
    dispatches lasting at least half the kernel's longest in that pass count."""
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "*", "pmc_counter_collection.csv")):
        rows = []
        for row in csv.DictReader(open(f)):
            name = next((v for k, v in KERNELS.items() if k in row["Kernel_Name"]), None)
            if name is not None:
                rows.append((name, int(row["End_Timestamp"]) - int(row["Start_Timestamp"]), row))
        longest = collections.defaultdict(int)
        for name, dur, _ in rows:
            longest[name] = max(longest[name], dur)
        for name, dur, row in rows:
            if dur * 2 >= longest[name]:
                acc[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--json", help="pmc_windows.json to update (entry keyed by --config)")
    ap.add_argument("--config", default="C2")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--levels", type=int, default=24)
    ap.add_argument("--calib", help="profiles/calib fetch_calib JSON lines: the Infinity-Cache gather "
                                    "ceiling (k_mall_sparse) for fabric_frac")
    ap.add_argument("--calib-pmc", help="the calibration run's PMC csv (TCC hit rate of k_mall_sparse)")
    a = ap.parse_args()
    res = load(a.dir)
    for k, cs in sorted(res.items()):
        print(k)
        for c, v in sorted(cs.items()):
            print("   %-36s %.6g" % (c, v))
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            hbm = (2 * cs["FETCH_SIZE"] + cs["WRITE_SIZE"]) * 1024
            print("   %-36s %.6g" % ("hbm_bytes_per_launch", hbm))
    if a.json and "windows" in res:
        cs = res["windows"]
        out = {"config": a.config, "batch": a.batch, "width": a.width, "height": a.height, "levels": a.levels,
               "source": a.dir, "counters_per_launch": cs,
               "hbm_bytes_per_launch": (2 * cs["FETCH_SIZE"] + cs["WRITE_SIZE"]) * 1024,
               "valu_insts_per_launch": cs.get("SQ_INSTS_VALU"),
               "note": "FETCH_SIZE doubled: it counts 64 B per 128-B L2 line fill, for coalesced "
                       "streams and 16-B-per-lane gathers alike (profiles/calib: k_stream, k_sparse, "
                       "k_dense8 each read lines x 64 B); KiB units"}
        if a.calib:
            for line in open(a.calib):
                d = json.loads(line)
                if d["kernel"] == "k_mall_sparse":
                    ceil = d["lines_per_s"]
                if d["kernel"] == "k_sparse":  # one pass over 1 GiB, cold: every line from HBM
                    out["hbm_gather_ceiling_lines_per_s"] = d["lines_per_s"]
            hit = 0.0
            if a.calib_pmc:
                h = m = 0.0
                for row in csv.DictReader(open(a.calib_pmc)):
                    if "k_mall_sparse" in row["Kernel_Name"]:
                        if row["Counter_Name"] == "TCC_HIT_sum":
                            h += float(row["Counter_Value"])
                        elif row["Counter_Name"] == "TCC_MISS_sum":
                            m += float(row["Counter_Value"])
                hit = h / (h + m) if h + m else 0.0
            # beyond-L2 lines per second the fabric delivered in the calibration
            out["fabric_ceiling_lines_per_s"] = ceil * (1.0 - hit)
            out["fabric_ceiling_source"] = ("profiles/calib k_mall_sparse: 16-B-per-lane gathers, one per "
                                            "128-B line, 64 MiB Infinity-Cache-resident table; requested "
                                            "lines/s x (1 - its L2 hit rate %.3f)" % hit)
        doc = {}
        if os.path.exists(a.json):
            doc = json.load(open(a.json))
            if "configs" not in doc:
                doc = {"configs": {doc.get("config", "C2"): doc}}
        doc.setdefault("configs", {})[a.config] = out
        json.dump(doc, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
