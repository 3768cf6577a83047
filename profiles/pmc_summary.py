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
import re

KERNELS = {"window_kernel": "windows", "cascade_kernel": "windows", "chain_kernel": "windows",
           "walk_kernel": "walk",
           "rowscan_kernel": "rowscan", "colscan_kernel": "colscan",
           "rowcarry_kernel": "rowscan", "colstrip_kernel": "colscan"}


def load(d):
    """Per kernel and counter, the mean over the batch's launches.  A pass may
    also hold launches of another shape (a batch-1 leg, a chunk tail): only
    dispatches lasting at least half the kernel's longest in that pass count."""
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    # rocprofv3 output dirs (PASS/pmc_counter_collection.csv), or the committed
    # copies of their counter files (PASS.csv)
    files = glob.glob(os.path.join(d, "*", "pmc_counter_collection.csv")) or \
        [f for f in glob.glob(os.path.join(d, "*.csv")) if "Counter_Name" in open(f).readline()]
    for f in files:
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
                acc[name]["_dispatch_ms"].append(dur / 1e6)
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


def build_id(d):
    """The library build id (sc_build_info) of the bench.py runs the passes
    profiled (their JSON lines' "build", profiles/collect_pmc_cfg.sh): one
    value, or an error."""
    ids = set()
    for f in glob.glob(os.path.join(d, "*.json")):
        try:
            line = json.loads(open(f).read().strip().splitlines()[-1])
        except (ValueError, IndexError):
            continue
        if "build" in line:
            ids.add(line["build"]["build_id"])
    if len(ids) != 1:
        raise SystemExit("%s: expected one build_id over the passes, found %s" % (d, sorted(ids)))
    return ids.pop()


# MI355X_MICROARCH.md (section "Indexed rows: gather into LDS"): 1,152-B rows
# gathered into LDS from a 38 MB Infinity-Cache-resident table, 8.6 TB/s --
# the best gather rate the guide measured beyond the L2
GUIDE_GATHER_LDS_BPS = 8.6e12


def ceilings(calib, calib_pmc=None):
    """Beyond-L2 gather ceilings (lines/s).  Measured: profiles/calib
    fetch_calib's gather kernels (k_rows*, k_mall_*: 1-KiB row pieces through
    LDS, 16-B-per-lane gathers), requested lines/s x (1 - L2 hit rate) -- the
    hit rate from the calibration run's TCC_HIT / TCC_MISS (calib_pmc) when
    given, else 4 MiB / T for a T-MiB table.  The fabric ceiling is the
    larger of the best measured rate (tables <= 256 MiB) and the guide's 8.6
    TB/s; nothing the chain kernel reaches may exceed it (it did exceed the
    round-3 same-shape figure at C4)."""
    import collections
    hit = {}
    if calib_pmc:
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for row in csv.DictReader(open(calib_pmc)):
            per[(row["Kernel_Name"].split("(")[0].strip(), row["Dispatch_Id"])][row["Counter_Name"]] += \
                float(row["Counter_Value"])
        by_kernel = collections.defaultdict(list)
        for (name, did), c in sorted(per.items(), key=lambda kv: int(kv[0][1])):
            if c.get("TCC_HIT_sum", 0) + c.get("TCC_MISS_sum", 0) > 0:
                by_kernel[name].append(c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"]))
        # k_mall_*: one table (64 MiB); k_rows / k_rows_dma: one warm + 4 timed
        # dispatches per table size, in fetch_calib's order
        for name, v in by_kernel.items():
            if name.startswith("k_rows"):
                for i, t in enumerate((32, 64, 256, 1024)):
                    if len(v) >= 5 * (i + 1):
                        hit["%s_%dMiB" % (name, t)] = min(v[5 * i:5 * i + 5])
            else:
                hit[name] = min(v)
    best, best_k, hbm = 0.0, None, None
    for line in open(calib):
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        k = d["kernel"]
        m = re.search(r"(\d+)MiB$", k)
        t_mib = int(m.group(1)) if m else (64 if k.startswith("k_mall") else None)
        if t_mib is None:
            continue
        h = hit.get(k, 4.0 / t_mib)
        beyond = d["lines_per_s"] * (1.0 - h)
        if t_mib <= 256 and beyond > best:
            best, best_k = beyond, k
        if t_mib > 256 and k.startswith("k_rows"):
            hbm = max(hbm or 0.0, beyond)
    guide = GUIDE_GATHER_LDS_BPS / 128.0
    return {"fabric_ceiling_lines_per_s": max(best, guide), "fabric_ceiling_measured_lines_per_s": best,
            "hbm_gather_ceiling_lines_per_s": hbm,
            "fabric_ceiling_source": "max(MI355X_MICROARCH.md gather-into-LDS 8.6 TB/s = %.3g lines/s, best "
                                     "measured beyond-L2 gather %.3g lines/s (%s, %s))"
                                     % (guide, best, best_k, calib)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--json", help="pmc_windows.json to update (entry keyed by --config)")
    ap.add_argument("--config", default="C2")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--levels", type=int, default=24)
    ap.add_argument("--calib", help="profiles/calib fetch_calib output (k_rows_* lines): the beyond-L2 "
                                    "gather ceilings for fabric_frac (stored top-level in the JSON)")
    ap.add_argument("--calib-pmc", help="the calibration run's pmc_counter_collection.csv (TCC hit rates)")
    a = ap.parse_args()
    res = load(a.dir)
    for k, cs in sorted(res.items()):
        print(k)
        for c, v in sorted(cs.items()):
            print("   %-36s %.6g" % (c, v))
        if k == "windows":
            print("   build_id", build_id(a.dir))
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            hbm = (2 * cs["FETCH_SIZE"] + cs["WRITE_SIZE"]) * 1024
            print("   %-36s %.6g" % ("hbm_bytes_per_launch", hbm))
    if a.json and "windows" in res:
        cs = dict(res["windows"])
        ms = cs.pop("_dispatch_ms", None)
        out = {"config": a.config, "batch": a.batch, "width": a.width, "height": a.height, "levels": a.levels,
               "source": a.dir, "build_id": build_id(a.dir), "counters_per_launch": cs,
               "avg_launch_ms_pmc": ms,
               "hbm_bytes_per_launch": (2 * cs["FETCH_SIZE"] + cs["WRITE_SIZE"]) * 1024,
               "valu_insts_per_launch": cs.get("SQ_INSTS_VALU"),
               "note": "FETCH_SIZE doubled: it counts 64 B per 128-B L2 line fill, for coalesced "
                       "streams and 16-B-per-lane gathers alike (profiles/calib: k_stream, k_sparse, "
                       "k_dense8 each read lines x 64 B); KiB units"}
        doc = {}
        if os.path.exists(a.json):
            doc = json.load(open(a.json))
            if "configs" not in doc:
                doc = {"configs": {doc.get("config", "C2"): doc}}
        if a.calib:
            doc["ceilings"] = ceilings(a.calib, a.calib_pmc)
        doc.setdefault("configs", {})[a.config] = out
        json.dump(doc, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
