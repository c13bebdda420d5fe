"""The gather probe's access-mix cases (scripts/td_probe --mix) with their
counter passes: per case the timed wave-load instruction rate, TD / TA busy,
L1 accesses per instruction, wait-any per wave cycle and L2 hit -- and TD busy
per unit of instruction rate (busy / (rate / the independent hot case's
rate)), the figure that tells whether dependent chains and L2 misses hold the
data-return unit longer per instruction, as the bounce kernel's 44% TD at 19%
of the independent-gather peak suggests.

    python scripts/td_mix_summary.py gpurun_out/r05n --json profiles/r05_td_mix.json
    (or the committed copy: profiles/r05_logs/r05n)
"""
import argparse
import collections
import csv
import json
import os
import statistics

CUS, XCDS = 256, 8


def dispatches(root):
    rows = []
    for dp, _, fs in os.walk(root):
        for f in fs:
            if f.endswith("counter_collection.csv"):
                rows += list(csv.DictReader(open(os.path.join(dp, f))))
    return per_dispatch(rows)


def dispatches_file(path):
    return per_dispatch(list(csv.DictReader(open(path)))) if os.path.exists(path) else []


def per_dispatch(rows):
    per = collections.defaultdict(dict)
    for r in rows:
        if "probe_mix" not in r["Kernel_Name"]:
            continue
        per[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    return [per[k] for k in sorted(per)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--json")
    a = ap.parse_args()
    txt = open(os.path.join(a.out, "mix.json")).read()
    probe = json.loads(txt[txt.index("{"):])
    cases = probe["cases"]
    # gpurun_out/<tag>/pmc.i/ (rocprofv3 -d) or the committed copy pmc.i.counter_collection.csv
    passes = [dispatches(os.path.join(a.out, f"pmc.{i}")) if os.path.isdir(os.path.join(a.out, f"pmc.{i}"))
              else dispatches_file(os.path.join(a.out, f"pmc.{i}.counter_collection.csv")) for i in range(1, 5)]
    for p_i, d in enumerate(passes):
        per_case = len(d) // len(cases) if d else 0
        for i, c in enumerate(cases):
            timed = [d[i * per_case + j] for j in range(1, per_case, 2)] if per_case else []
            if not timed:
                continue
            med = lambda k: statistics.median(x[k] for x in timed if k in x)  # noqa: E731
            if "GRBM_GUI_ACTIVE" in timed[0]:
                g = med("GRBM_GUI_ACTIVE") / XCDS
                c["kernel_ms_at_2400MHz"] = round(g / 2.4e6, 4)
                if "TD_TD_BUSY_sum" in timed[0]:
                    c["td_busy"] = round(med("TD_TD_BUSY_sum") / (CUS * g), 4)
                if "TA_TA_BUSY_sum" in timed[0]:
                    c["ta_busy"] = round(med("TA_TA_BUSY_sum") / (CUS * g), 4)
            if "SQ_INSTS_VMEM_RD" in timed[0]:
                c["tcp_accesses_per_instruction"] = round(med("TCP_TOTAL_CACHE_ACCESSES_sum") / med("SQ_INSTS_VMEM_RD"), 3)
                c["wait_any_per_wave_cycle"] = round(med("SQ_WAIT_ANY") / med("SQ_WAVE_CYCLES"), 4)
                if "SQ_INSTS_VALU" in timed[0]:
                    c["valu_per_vmem_rd"] = round(med("SQ_INSTS_VALU") / med("SQ_INSTS_VMEM_RD"), 2)
                    c["lds_per_vmem_rd"] = round(med("SQ_INSTS_LDS") / med("SQ_INSTS_VMEM_RD"), 3)
            if "TCC_HIT_sum" in timed[0]:
                h, mi = med("TCC_HIT_sum"), med("TCC_MISS_sum")
                c["l2_hit"] = round(h / max(h + mi, 1.0), 4)
    base = next((c for c in cases if c["dependent"] == 0 and c["cold_frac"] == 0 and c["active_lanes"] == 20
                 and not c.get("valu_fma_per_visit") and not c.get("lds_reads_per_visit")
                 and not c.get("dword_loads_per_visit")), None)
    for c in cases:
        if base and "td_busy" in c:
            rel = c["ginst_per_s"] / base["ginst_per_s"]
            c["rate_vs_independent_hot"] = round(rel, 4)
            c["td_busy_per_rate"] = round(c["td_busy"] / max(rel, 1e-9), 4)
        print(json.dumps(c))
    if a.json:
        probe["method"] = __doc__.strip().split("\n\n")[0]
        with open(a.json, "w") as f:
            json.dump(probe, f, indent=1)


if __name__ == "__main__":
    main()
