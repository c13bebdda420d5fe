"""The bounce launch of the timed shape ALONE under the kernel trace
(scripts/r04q_gpu.sh's prof_exclusive run: bench.py --pipeline 1
--bounce-blocks 384) against the counter pass's exclusive time: both must
agree for bench.py's roofline kernel_ms (trace_check).

    python scripts/exclusive_trace.py <rocprofv3 -d dir> <pmc bound json> <out json>
"""
import csv
import json
import os
import statistics
import sys


def main():
    d, pmc_path, out = sys.argv[1:4]
    grid = 384 * 256
    ms = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
          for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv")))
          if "bounce_kernel" in r["Kernel_Name"] and int(r["Grid_Size_X"]) == grid]
    pmc = json.load(open(pmc_path))
    res = {"command": "rocprofv3 --kernel-trace --stats -- python3 bench.py --no-cpu --no-host --pipeline 1 "
                      "--bounce-blocks 384 --steps 20 --warmup 5",
           "kernel": "bounce_kernel<true, 2, false>, grid 98304 work-items (384 workgroups: the timed launch shape), "
                     "one launch at a time",
           "dispatches": len(ms), "mean_ms": round(statistics.mean(ms), 4),
           "median_ms": round(statistics.median(ms), 4), "min_ms": round(min(ms), 4), "max_ms": round(max(ms), 4),
           "pmc_exclusive_ms": pmc["kernels"]["timed/bounce"]["vmem_pass"]["kernel_ms_at_2400MHz"],
           "pmc_source": pmc_path + " timed/bounce vmem_pass.kernel_ms_at_2400MHz"}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
