"""The exclusive-time check of bench.py's roofline (kernel_ms_trace_check):
the bounce launches of the timed shape (384 workgroups) run ONE at a time
under rocprofv3 --kernel-trace, their mean duration beside the counter pass's
exclusive time.

    rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/<tag>/prof_exclusive -o run -- \
        python3 bench.py --no-cpu --no-host --pipeline 1 --bounce-blocks 384 --steps 20 --warmup 5
    python scripts/exclusive_trace.py gpurun_out/<tag>/prof_exclusive/run_kernel_trace.csv \
        --pmc profiles/r05_pmc_bound_1080p_10k.json --json profiles/r05_exclusive_bounce_trace.json
"""
import argparse
import csv
import json
import statistics

BOUNCE = "bounce_kernel<true, 2, false>"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--pmc", required=True)
    ap.add_argument("--grid", type=int, default=384 * 256)
    ap.add_argument("--json")
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.trace)) if BOUNCE in r["Kernel_Name"] and int(r["Grid_Size_X"]) == a.grid]
    ms = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
    pmc = json.load(open(a.pmc))
    out = {"command": "rocprofv3 --kernel-trace --stats -- python3 bench.py --no-cpu --no-host --pipeline 1 "
                      "--bounce-blocks 384 --steps 20 --warmup 5",
           "kernel": f"{BOUNCE}, grid {a.grid} work-items (384 workgroups: the timed launch shape), one launch at "
                     "a time",
           "dispatches": len(ms), "mean_ms": round(statistics.mean(ms), 4), "median_ms": round(statistics.median(ms), 4),
           "min_ms": round(min(ms), 4), "max_ms": round(max(ms), 4),
           "pmc_exclusive_ms": pmc["kernels"]["timed/bounce"]["vmem_pass"]["kernel_ms_at_2400MHz"],
           "pmc_source": a.pmc + " timed/bounce vmem_pass.kernel_ms_at_2400MHz"}
    print(json.dumps(out))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
