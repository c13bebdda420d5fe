"""Summarise scripts/pmc_probe.sh output into the bound of each frame kernel.

    python scripts/pmc_summary.py gpurun_out/<tag> [--json profiles/<tag>_pmc_bound.json] [--copy profiles/<tag>_pmc]

Per config and kernel (primary / bounce): the median over its launches of
every counter (the first launch of a run is cold, the median ignores it), and
the utilisations derived from them (MI355X_MICROARCH.md for the units):

  kernel cycles     GRBM_GUI_ACTIVE / 8 (the counter sums the 8 XCDs)
  TD / TA busy      TD_TD_BUSY_sum, TA_TA_BUSY_sum over 256 CUs x cycles
  VALU busy         SQ_INSTS_VALU x 2 cycles (one wave64 instruction issues over
                    2 cycles) over 1024 SIMDs x cycles
  L2 hit            TCC_HIT / (TCC_HIT + TCC_MISS)
  L2 read bytes     TCP_TCC_READ_REQ x 128 B (gfx950 L2 line; an upper bound:
                    partial-line requests count as whole lines) vs the 34.5 TB/s L2
  L1 accesses       TCP_TOTAL_CACHE_ACCESSES per CU per cycle
  HBM bytes         FETCH_SIZE x 2 (gfx950 tallies a wide read at half) +
                    WRITE_SIZE, both KiB
  mean L2 latency   TCP_TCC_READ_REQ_LATENCY / TCP_TCC_READ_REQ (cycles)
  vmem_pass         from the ONE pass holding SQ_INSTS_VMEM_RD, GRBM_GUI_ACTIVE and
                    TCP_TOTAL_CACHE_ACCESSES_sum: the kernel's wave-level load
                    instructions, its exclusive time and its L1 accesses per load
                    instruction (bench.py's roofline: / the gather peak of the same
                    access shape, profiles/r04_td_probe.json)
"""
import argparse
import collections
import csv
import glob
import json
import os
import shutil
import statistics

CLOCK_HZ = 2.4e9
CUS, SIMDS, XCDS = 256, 1024, 8
L2_PEAK_GBS = 34500.0
HBM_PEAK_GBS = 8000.0


def kernel_of(name):
    if "bounce_kernel" in name:
        return "bounce"
    if "primary_kernel" in name:
        return "primary"
    return None


def derive(c):
    d = {}
    g = c.get("GRBM_GUI_ACTIVE", 0) / XCDS
    if not g:
        return d
    d["kernel_cycles"] = int(g)
    d["kernel_ms_at_2400MHz"] = round(g / CLOCK_HZ * 1e3, 4)
    sec = g / CLOCK_HZ
    if "TD_TD_BUSY_sum" in c:
        d["td_busy"] = round(c["TD_TD_BUSY_sum"] / (CUS * g), 4)
    if "TA_TA_BUSY_sum" in c:
        d["ta_busy"] = round(c["TA_TA_BUSY_sum"] / (CUS * g), 4)
    if "SQ_INSTS_VALU" in c:
        d["valu_busy"] = round(c["SQ_INSTS_VALU"] * 2 / (SIMDS * g), 4)
    if "SQ_WAVE_CYCLES" in c:
        wc = c["SQ_WAVE_CYCLES"]
        d["wait_any_per_wave_cycle"] = round(c["SQ_WAIT_ANY"] / wc, 4)
        d["wait_inst_any_per_wave_cycle"] = round(c["SQ_WAIT_INST_ANY"] / wc, 4)
        d["active_inst_any_per_wave_cycle"] = round(c["SQ_ACTIVE_INST_ANY"] / wc, 4)
    if "TCC_HIT_sum" in c:
        d["l2_hit"] = round(c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"]), 4)
    if "TCP_TCC_READ_REQ_sum" in c:
        b = c["TCP_TCC_READ_REQ_sum"] * 128
        d["l2_read_bytes_upper"] = int(b)
        d["l2_read_gbs_upper"] = round(b / sec / 1e9, 1)
        d["l2_frac_upper"] = round(b / sec / 1e9 / L2_PEAK_GBS, 4)
    if "TCP_TOTAL_CACHE_ACCESSES_sum" in c:
        d["l1_accesses_per_cu_cycle"] = round(c["TCP_TOTAL_CACHE_ACCESSES_sum"] / (CUS * g), 4)
    if "TCP_TCC_READ_REQ_LATENCY_sum" in c and c.get("TCP_TCC_READ_REQ_sum"):
        d["l2_read_latency_cycles"] = round(c["TCP_TCC_READ_REQ_LATENCY_sum"] / c["TCP_TCC_READ_REQ_sum"], 1)
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        b = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
        d["hbm_bytes"] = int(b)
        d["hbm_gbs"] = round(b / sec / 1e9, 2)
        d["hbm_frac"] = round(b / sec / 1e9 / HBM_PEAK_GBS, 5)
    units = {k: d[k] for k in ("td_busy", "ta_busy", "valu_busy", "l2_frac_upper", "hbm_frac") if k in d}
    if units:
        top = max(units, key=units.get)
        d["busiest_unit"] = top
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--json")
    ap.add_argument("--copy", help="copy the raw counter CSVs here")
    ap.add_argument("--workload", default="1920,1080,10000,5",
                    help="W,H,spheres,depth the probe rendered (scripts/profile_kernel.py defaults)")
    ap.add_argument("--pattern", default="t*_f*_d*.*",
                    help="pass directories (scripts/pmc_probe.sh: t*_f*_d*.N; scripts/pmc_bench.sh: bench.N)")
    ap.add_argument("--bounce-grid", type=int, default=0,
                    help="count only bounce dispatches of this many work-items (the timed loop's launch shape)")
    ap.add_argument("--name", default=None, help="config name for the output keys (default: the directory stem)")
    a = ap.parse_args()
    cfgs = collections.defaultdict(dict)
    for d in sorted(glob.glob(os.path.join(a.root, a.pattern))):
        if d.endswith(".log"):
            continue
        cfg = a.name or os.path.basename(d).rsplit(".", 1)[0]
        f = os.path.join(d, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        if a.copy:
            os.makedirs(a.copy, exist_ok=True)
            shutil.copy(f, os.path.join(a.copy, os.path.basename(d) + ".csv"))
        acc = collections.defaultdict(list)
        names = {}
        for r in csv.DictReader(open(f)):
            kern = kernel_of(r["Kernel_Name"])
            if kern == "bounce" and a.bounce_grid and int(r["Grid_Size"]) != a.bounce_grid:
                continue
            if kern:
                acc[(kern, r["Counter_Name"])].append(float(r["Counter_Value"]))
                names[kern] = r["Kernel_Name"]
        for (kern, k), v in acc.items():
            e = cfgs[cfg + "/" + kern]
            e.setdefault("_all", collections.defaultdict(list))[k] += v
            # each pass on its own too: values that must come from ONE pass
            # (the vmem roofline: instructions, time and access shape) are
            # read from the pass that holds SQ_INSTS_VMEM_RD
            e.setdefault("passes", {}).setdefault(os.path.basename(d), {})[k] = statistics.median(v)
            e["kernel"] = names[kern]
    for e in cfgs.values():
        allv = e.pop("_all")
        e["counters"] = {k: statistics.median(v) for k, v in allv.items()}
        e["launches"] = {k: len(v) for k, v in allv.items()}
    out = {}
    for cfg, e in sorted(cfgs.items()):
        e["derived"] = derive(e["counters"])
        vp = [p for p in e.get("passes", {}).values() if "SQ_INSTS_VMEM_RD" in p and "GRBM_GUI_ACTIVE" in p]
        if vp:
            p = vp[0]
            g = p["GRBM_GUI_ACTIVE"] / XCDS
            e["vmem_pass"] = {
                "SQ_INSTS_VMEM_RD": p["SQ_INSTS_VMEM_RD"], "GRBM_GUI_ACTIVE": p["GRBM_GUI_ACTIVE"],
                "TCP_TOTAL_CACHE_ACCESSES_sum": p.get("TCP_TOTAL_CACHE_ACCESSES_sum"), "SQ_WAVES": p.get("SQ_WAVES"),
                "kernel_ms_at_2400MHz": round(g / CLOCK_HZ * 1e3, 4),
                "vmem_ginst_per_s": round(p["SQ_INSTS_VMEM_RD"] / (g / CLOCK_HZ) / 1e9, 3),
                "tcp_accesses_per_instruction": round(p["TCP_TOTAL_CACHE_ACCESSES_sum"] / p["SQ_INSTS_VMEM_RD"], 3)
                if p.get("TCP_TOTAL_CACHE_ACCESSES_sum") else None}
        out[cfg] = e
        print(cfg, e["kernel"][:80])
        for k, v in sorted(e["derived"].items()):
            print(f"   {k:34s} {v}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"source": f"{'scripts/pmc_bench.sh' if a.pattern.startswith('bench') else 'scripts/pmc_probe.sh'}"
                                 f" -> {a.root}" + (f" (bounce dispatches of {a.bounce_grid} work-items)"
                                                    if a.bounce_grid else ""), "clock_hz": CLOCK_HZ,
                       "workload": [int(v) for v in a.workload.split(",")],
                       "l2_peak_gbs": L2_PEAK_GBS, "hbm_peak_gbs": HBM_PEAK_GBS,
                       "method": __doc__.strip().split("\n\n", 2)[-1], "kernels": out}, f, indent=1)


if __name__ == "__main__":
    main()
