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
                acc[name]["_dispatch_ms"].append(dur / 1e6)
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


def sources_sha(d):
    """kernel_sources_sha of the bench.py runs the passes profiled (their JSON
    lines, profiles/collect_pmc_cfg.sh): one value, or an error."""
    shas = set()
    for f in glob.glob(os.path.join(d, "*.json")):
        try:
            line = json.loads(open(f).read().strip().splitlines()[-1])
        except (ValueError, IndexError):
            continue
        if "kernel_sources_sha" in line:
            shas.add(line["kernel_sources_sha"])
    if len(shas) != 1:
        raise SystemExit("%s: expected one kernel_sources_sha over the passes, found %s" % (d, sorted(shas)))
    return shas.pop()


def ceilings(calib):
    """Beyond-L2 gather ceilings from profiles/calib fetch_calib's k_rows_<T>MiB
    lines (1-KiB row pieces through LDS, MI355X_MICROARCH.md's best gather
    form): requested lines/s x (1 - 4 MiB / T), the share of a uniformly
    gathered table an XCD's L2 holds; the fabric ceiling is the best table
    that fits the Infinity Cache, the HBM one the 1 GiB table."""
    fab, hbm = None, None
    for line in open(calib):
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        if not d["kernel"].startswith("k_rows_"):
            continue
        t_mib = int(re.search(r"(\d+)MiB$", d["kernel"]).group(1))
        beyond = d["lines_per_s"] * (1.0 - 4.0 / t_mib)
        if t_mib <= 256:
            fab = max(fab or 0.0, beyond)
        else:
            hbm = beyond
    return {"fabric_ceiling_lines_per_s": fab, "hbm_gather_ceiling_lines_per_s": hbm,
            "fabric_ceiling_source": "profiles/calib k_rows_<T>MiB (%s): 1-KiB random row pieces staged "
                                     "through LDS, requested lines/s x (1 - 4 MiB/T); fabric = best T <= "
                                     "256 MiB, HBM = 1 GiB" % calib}


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
    a = ap.parse_args()
    res = load(a.dir)
    for k, cs in sorted(res.items()):
        print(k)
        for c, v in sorted(cs.items()):
            print("   %-36s %.6g" % (c, v))
        if k == "windows":
            print("   kernel_sources_sha", sources_sha(a.dir))
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            hbm = (2 * cs["FETCH_SIZE"] + cs["WRITE_SIZE"]) * 1024
            print("   %-36s %.6g" % ("hbm_bytes_per_launch", hbm))
    if a.json and "windows" in res:
        cs = dict(res["windows"])
        ms = cs.pop("_dispatch_ms", None)
        out = {"config": a.config, "batch": a.batch, "width": a.width, "height": a.height, "levels": a.levels,
               "source": a.dir, "kernel_sources_sha": sources_sha(a.dir), "counters_per_launch": cs,
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
            doc["ceilings"] = ceilings(a.calib)
        doc.setdefault("configs", {})[a.config] = out
        json.dump(doc, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
