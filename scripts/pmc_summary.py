"""Summarise scripts/pmc_probe.sh output: per config, the render kernel's
counters (median over its launches)."""
import collections
import csv
import glob
import os
import statistics
import sys

root = sys.argv[1]
cfgs = collections.defaultdict(dict)
for d in sorted(glob.glob(os.path.join(root, "t*_f*_d*.*"))):
    if d.endswith(".log"):
        continue
    cfg = os.path.basename(d).rsplit(".", 1)[0]
    f = os.path.join(d, "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        kern = ("bounce" if "bounce_kernel" in name else "primary" if "primary_kernel" in name else
                "render" if "render_kernel" in name and "true, true" not in name else None)
        if kern:
            acc[(kern, r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (kern, k), v in acc.items():
        cfgs[cfg + "/" + kern][k] = statistics.median(v)
for cfg, c in cfgs.items():
    g = c.get("GRBM_GUI_ACTIVE", 0) / 8
    print(cfg, "kernel_cycles(per XCD)", int(g))
    for k in sorted(c):
        print(f"   {k:40s} {c[k]:.4g}")
    if g and "SQ_WAVE_CYCLES" in c:
        wc = c["SQ_WAVE_CYCLES"]
        print("   derived: WAIT_ANY/WAVE %.2f  WAIT_INST/WAVE %.2f  ACTIVE/WAVE %.2f" % (
            c["SQ_WAIT_ANY"] / wc, c["SQ_WAIT_INST_ANY"] / wc, c["SQ_ACTIVE_INST_ANY"] / wc))
        print("   derived: VALU busy per SIMD %.3f" % (c["SQ_INSTS_VALU"] * 2 / (g * 1024)))
    if "TCC_HIT_sum" in c:
        print("   derived: L2 hit %.3f  TA busy frac %.3f" % (
            c["TCC_HIT_sum"] / max(1, c["TCC_HIT_sum"] + c["TCC_MISS_sum"]), c.get("TA_TA_BUSY_sum", 0) / max(1, g * 256)))
    if "TCP_TOTAL_CACHE_ACCESSES_sum" in c:
        print("   derived: L1 miss->L2 requests / accesses %.3f" % (
            c["TCP_TCC_READ_REQ_sum"] / max(1, c["TCP_TOTAL_CACHE_ACCESSES_sum"])))
