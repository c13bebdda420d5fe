"""Combine scripts/td_probe's timed output with its counter passes into the
gather-peak table bench.py prices the bounce kernel against
(profiles/r04_td_probe.json).

    python scripts/td_probe_summary.py gpurun_out/r04a/td_probe.log \
        gpurun_out/r04a/td_pmc_acc gpurun_out/r04a/td_pmc_busy --json profiles/r04_td_probe.json

Per probe case (nodes touched per wave-load instruction): the timed chip rate
of wave-level dwordx4 loads (G instructions/s), and from the counter passes
(the probe's dispatches in order: 3 x (warm-up, timed) per case, the timed
launches' median) the L1 (TCP) accesses per load instruction and the TA / TD
busy fractions -- the last show which unit a fully divergent gather
saturates. bench.py looks up the bounce kernel's own TCP accesses per load
instruction in this table (linear interpolation over the accesses) to get
the peak rate of the same access shape.
"""
import argparse
import collections
import csv
import json
import os
import statistics

CUS, XCDS = 256, 8


def dispatches(root):
    f = os.path.join(root, "run_counter_collection.csv")
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(f)):
        if "probe" not in r["Kernel_Name"]:
            continue
        per[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    return [per[k] for k in sorted(per)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("timed")
    ap.add_argument("acc")
    ap.add_argument("busy")
    ap.add_argument("--json")
    a = ap.parse_args()
    txt = open(a.timed).read()
    probe = json.loads(txt[txt.index("{"):])
    cases = probe["cases"]
    acc, busy = dispatches(a.acc), dispatches(a.busy)
    per_case = len(acc) // len(cases)
    for i, c in enumerate(cases):
        timed_acc = [acc[i * per_case + j] for j in range(1, per_case, 2)]
        timed_busy = [busy[i * per_case + j] for j in range(1, per_case, 2)]
        g = statistics.median(d["GRBM_GUI_ACTIVE"] for d in timed_busy) / XCDS
        c["tcp_accesses_per_instruction"] = round(statistics.median(
            d["TCP_TOTAL_CACHE_ACCESSES_sum"] / d["SQ_INSTS_VMEM_RD"] for d in timed_acc), 3)
        c["vmem_rd_per_launch"] = statistics.median(d["SQ_INSTS_VMEM_RD"] for d in timed_acc)
        c["td_busy"] = round(statistics.median(d["TD_TD_BUSY_sum"] for d in timed_busy) / (CUS * g), 4)
        c["ta_busy"] = round(statistics.median(d["TA_TA_BUSY_sum"] for d in timed_busy) / (CUS * g), 4)
    probe["per_case_dispatches"] = per_case
    probe["method"] = __doc__.strip().split("\n\n", 2)[-1]
    for c in cases:
        print(f"nodes/inst {c['nodes_per_instruction']:2d}  lanes/node {c['lanes_per_node']:2d}  "
              f"{c['ginst_per_s']:8.2f} Ginst/s  {c['cycles_per_instruction_per_cu']:6.2f} cyc/inst/CU  "
              f"TCP/inst {c['tcp_accesses_per_instruction']:6.2f}  TD {c['td_busy']:.3f}  TA {c['ta_busy']:.3f}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(probe, f, indent=1)


if __name__ == "__main__":
    main()
