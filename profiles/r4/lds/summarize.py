"""Per-kernel PMC of itembench V0 (production gathers) vs V14 (every corner an
LDS read): profiles/r4/lds/pmc_{sq,td}_{0,14}_16 -> summary.txt."""
import collections
import csv
import os

D = os.path.dirname(os.path.abspath(__file__))
out = []
for n, kname in (("0_16", "k_base"), ("14_16", "k_ldsgather")):
    agg, dur = collections.defaultdict(float), None
    for kind in ("sq", "td"):
        for r in csv.DictReader(open(os.path.join(D, "pmc_%s_%s" % (kind, n), "pmc_counter_collection.csv"))):
            if kname in r["Kernel_Name"]:
                agg[r["Counter_Name"]] += float(r["Counter_Value"])
    for r in csv.DictReader(open(os.path.join(D, "pmc_td_%s" % n, "pmc_kernel_trace.csv"))):
        if kname in r["Kernel_Name"]:
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    cyc = agg["GRBM_GUI_ACTIVE"] / 8  # per-XCD busy cycles of the dispatch
    out.append("%-11s %.3f ms  VMEM_RD %.3g  LDS insts %.3g  VALU %.3g" % (kname, dur, agg["SQ_INSTS_VMEM_RD"],
                                                                          agg["SQ_INSTS_LDS"], agg["SQ_INSTS_VALU"]))
    out.append("   TD busy / cycles %.3f   TD transfer (16 cyc x VMEM_RD) / cycles %.3f   LDS-active / cycles %.3f"
               "   bank-conflict cycles / LDS-active %.3f   VALU / (2 per CU-cycle) %.3f   wait / wave-cycles %.3f"
               % (agg["TD_TD_BUSY_sum"] / 256 / cyc, agg["SQ_INSTS_VMEM_RD"] * 16 / 256 / cyc,
                  agg["SQ_LDS_IDX_ACTIVE"] / 256 / cyc, agg["SQ_LDS_BANK_CONFLICT"] / agg["SQ_LDS_IDX_ACTIVE"],
                  agg["SQ_INSTS_VALU"] / (1024 * 0.5 * cyc), agg["SQ_WAIT_ANY"] / agg["SQ_WAVE_CYCLES"]))
open(os.path.join(D, "summary.txt"), "w").write("\n".join(out) + "\n")
print("\n".join(out))
