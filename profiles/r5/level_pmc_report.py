"""Per level range: the chain kernel's counters per launch (profiles/r5/
level_pmc.sh passes), time per launch, L2 hit, beyond-L2 lines/s against the
fabric ceiling (profiles/pmc_windows.json "ceilings"), texture-data-path busy
and load instructions per weak evaluation (items from
profiles/r4/items_per_level.json when the config's levels are there).

    python profiles/r5/level_pmc_report.py OUTDIR [--config C2] [--json out.json]
"""
import argparse
import glob
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import pmc_summary  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--config", default="C2")
    ap.add_argument("--frames", type=int, default=32)
    ap.add_argument("--json")
    a = ap.parse_args()
    pm = json.load(open(os.path.join(os.path.dirname(HERE), "pmc_windows.json")))
    ceil = pm.get("ceilings", {}).get("fabric_ceiling_lines_per_s")
    ipl = {}
    p = os.path.join(os.path.dirname(HERE), "r4", "items_per_level.json")
    if os.path.exists(p):
        ipl = json.load(open(p)).get(a.config, {})
    out = {}
    for d in sorted(glob.glob(os.path.join(a.dir, "*_*"))):
        if not os.path.isdir(d):
            continue
        lo, hi = (int(x) for x in os.path.basename(d).split("_"))
        c = pmc_summary.load(d).get("windows", {})
        if not c:
            continue
        ms = c.get("_dispatch_ms")
        s = ms / 1e3 if ms else None
        r = {"levels": [lo, hi], "chain_ms_pmc": ms, "counters_per_launch": c}
        hit, miss = c.get("TCC_HIT_sum"), c.get("TCC_MISS_sum")
        if hit and miss:
            r["l2_hit"] = hit / (hit + miss)
            r["beyond_l2_lines_per_s"] = miss / s
            if ceil:
                r["fabric_frac"] = miss / s / ceil
        cyc = c.get("GRBM_GUI_ACTIVE")
        if cyc:
            cx = cyc / 8.0
            if c.get("TD_TD_BUSY_sum"):
                r["td_busy_frac"] = c["TD_TD_BUSY_sum"] / (256 * cx)
            if c.get("SQ_INSTS_VMEM_RD"):
                r["td_transfer_frac"] = c["SQ_INSTS_VMEM_RD"] * 16 / (256 * cx)
        if c.get("TCP_TCC_READ_REQ_LATENCY_sum") and c.get("TCP_TCC_READ_REQ_sum"):
            r["l1_miss_latency_cycles"] = c["TCP_TCC_READ_REQ_LATENCY_sum"] / c["TCP_TCC_READ_REQ_sum"]
        items = [lv["items"] for lv in ipl.get("levels", [])]
        if len(items) >= hi and s:
            n = sum(items[lo:hi]) * a.frames
            r["weak_evals_per_launch"] = n
            r["ps_per_weak_eval"] = s / n * 1e12
            if c.get("SQ_INSTS_VMEM_RD"):
                r["vmem_rd_per_weak_eval_x64"] = c["SQ_INSTS_VMEM_RD"] * 64 / n
        out["%d:%d" % (lo, hi)] = r
        print("%5s-%-3d %8.3f ms  L2 hit %.3f  fabric %.3f  TD busy %.3f (transfer %.3f)  L1-miss lat %.0f  ps/eval %s"
              % (lo, hi, ms or 0, r.get("l2_hit", 0), r.get("fabric_frac", 0), r.get("td_busy_frac", 0),
                 r.get("td_transfer_frac", 0), r.get("l1_miss_latency_cycles", 0),
                 "%.1f" % r["ps_per_weak_eval"] if "ps_per_weak_eval" in r else "-"))
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
