"""The reference's benchmark mode (benchmark.c:283-332) on one MI355X, with
the reference itself (oracle/_ref, unmodified sources, one core as the
reference runs) timed on the same sweep beside it.

    python scripts/bench_mode.py [--seed 1] [--reps 5] [--no-cpu] [--data benchmark_data.txt]

Prints the reference's per-point report, then one JSON line per point:
GPU device seconds of each loop (HIP events, median of reps), the rate in
Mrays/s and in sphere tests/s, the hit counts (checked equal to the
reference's when the CPU leg runs), and the reference's clock() seconds.
"""
import argparse
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401  (one HIP runtime in the process: torch's, as in bench.py)

mirt = importlib.import_module("cs201_sah-bvh_ray_tracer_amd")
bm = importlib.import_module("cs201_sah-bvh_ray_tracer_amd.benchmark")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--rays", type=int, default=bm.NUM_RAYS)
    ap.add_argument("--counts", default=None, help="comma-separated sphere counts (default benchmark.c's sweep)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--data", default=None, help="append save_benchmark_data lines here")
    a = ap.parse_args()
    counts = [int(c) for c in a.counts.split(",")] if a.counts else bm.DEFAULT_COUNTS
    r = mirt.Renderer(0)
    rows = bm.run_benchmark(r, counts, a.rays, a.seed, reps=a.reps, data_path=a.data, verbose=True)
    ref = None
    if not a.no_cpu:
        from oracle.lib import Reference
        ref = Reference(160, 90)
        ref.srand(a.seed)
    for row in rows:
        n = row["spheres"]
        out = {k: v for k, v in row.items() if not k.startswith("hit_")}
        out["gpu_no_bvh_sphere_tests_per_s_G"] = round(row["tests"] / row["time_no_bvh_s"] / 1e9, 2)
        out["gpu_no_bvh_mrays_s"] = round(a.rays / row["time_no_bvh_s"] / 1e6, 2)
        out["gpu_bvh_mrays_s"] = round(a.rays / row["time_bvh_s"] / 1e6, 2)
        if ref is not None:
            p = ref.bench_point(n, a.rays)
            assert int(p["hit_no_bvh"].sum()) == row["hits_no_bvh"] and (p["hit_no_bvh"] == row["hit_no_bvh"]).all()
            assert int(p["hit_bvh"].sum()) == row["hits_bvh"] and (p["hit_bvh"] == row["hit_bvh"]).all()
            out["ref_cpu_1core_s"] = [round(v, 4) for v in p["secs"]]
            out["speedup_no_bvh"] = round(p["secs"][0] / row["time_no_bvh_s"], 1)
            out["speedup_bvh"] = round(p["secs"][1] / row["time_bvh_s"], 1) if p["secs"][1] > 0 else None
            out["hits_equal_reference"] = True
        print(json.dumps(out), flush=True)
    r.close()


if __name__ == "__main__":
    main()
