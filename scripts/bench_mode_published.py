"""The reference's benchmark mode (benchmark.c:283-332) at the sphere counts
of its ONLY published numbers: results/benchmark_data.txt:1-6, 1K .. 100M
spheres (the commented sweep of benchmark.c:296), 10,000 rays per loop
(benchmark.c:297), one glibc rand() stream over the whole sweep
(benchmark.c:287: srand once; seed fixed here), trees built as
benchmark.c:317 builds them (over [0, n - 1), from depth 20).

    python scripts/bench_mode_published.py [--out profiles/r03_bench_mode] [--check-rays 256]

Writes <out>_benchmark_data.txt ("n time_no_bvh time_with_bvh" in seconds,
save_benchmark_data's format, benchmark.c:160-170: the GPU's device times of
the two loops, HIP events, median of --reps) and <out>.json: per point the
GPU times, the published reference times beside them and their ratio, the
log-log slopes of results/main.py:48-50 for both, and the parity check --
for the first --check-rays rays of each loop, the GPU's any-hit flags
(brute force, every sphere) and closest-hit records (BVH) equal the
oracle's (oracle/: the CPU restatement, pinned to the reference; its BVH
check rebuilds the tree with its own build, up to --oracle-max-bvh spheres).
"""
import argparse
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401  (one HIP runtime in the process: torch's, as in bench.py)

mirt = importlib.import_module("cs201_sah-bvh_ray_tracer_amd")
bm = importlib.import_module("cs201_sah-bvh_ray_tracer_amd.benchmark")

# results/benchmark_data.txt:1-6 (seconds: brute force, BVH; hardware not stated)
PUBLISHED = {1000: (0.001316, 0.000108), 10000: (0.011460, 0.000416), 100000: (0.122593, 0.001274),
             1000000: (1.229925, 0.006040), 10000000: (12.314131, 0.012367), 100000000: (123.909577, 0.027767)}


def slope(n, t):
    return float(np.polyfit(np.log(np.asarray(n, float)), np.log(np.asarray(t, float)), 1)[0])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--rays", type=int, default=bm.NUM_RAYS)
    ap.add_argument("--counts", default=",".join(str(n) for n in PUBLISHED))
    ap.add_argument("--check-rays", type=int, default=256)
    ap.add_argument("--oracle-max-bvh", type=int, default=1000000)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r03_bench_mode"))
    a = ap.parse_args()
    counts = [int(c) for c in a.counts.split(",")]
    from oracle.lib import Oracle
    o = Oracle()
    r = mirt.Renderer(0)
    st = mirt.RandState(a.seed)
    rows = []
    for n in counts:
        t0 = time.perf_counter()
        pre = mirt.create_benchmark_spheres(n, world_size=bm.WORLD_SIZE, state=st)
        spheres = pre.copy()
        tree = mirt.build_bvh(spheres, 0, n - 1, 20)            # benchmark.c:317
        build_s = time.perf_counter() - t0
        rays_a = mirt.create_bench_rays(a.rays, st)               # benchmark.c:176-185
        rays_b = mirt.create_bench_rays(a.rays, st)               # benchmark.c:228-237
        r.upload(spheres, tree)
        hit_a, t_no, w_no = bm._timed(lambda: r.any_hit(rays_a, use_bvh=False), r, a.reps)
        hits_b, t_bvh, w_bvh = bm._timed(lambda: r.closest_hit(rays_b, use_bvh=True), r, a.reps)
        k = min(a.check_rays, a.rays)
        # parity: any-hit flags of the brute-force loop (every sphere, benchmark.c:190-205), on
        # as many rays as ~2e9 oracle sphere tests allow (single-threaded CPU)
        ka = min(k, max(8, int(2e9 // n)))
        ref_a = o.intersect(None, spheres, rays_a[:ka], use_bvh=False)
        ok_a = bool((ref_a["hit"] == hit_a[:ka]).all())
        # closest-hit records of the BVH loop (hit.c:91-109): up to --oracle-max-bvh
        # spheres on the oracle's own build of the tree; beyond, the oracle's DFS over
        # the product's flat tree (its build is pinned by the tree SHA tests)
        if n <= a.oracle_max_bvh:
            so = pre.copy()
            t = o.build(so, 0, n - 1, 20)
            ref_b = o.intersect(t, so, rays_b[:k])
            o.free(t)
            bvh_check = "oracle build + hit.c DFS"
        else:
            ref_b = o.intersect_flat(tree.nodes, spheres[:n - 1], rays_b[:k])
            bvh_check = "hit.c DFS over the product's flat tree"
        ok_b = ref_b.tobytes() == hits_b[:k].tobytes()
        pub = PUBLISHED.get(n)
        row = {"spheres": n, "rays": a.rays, "bvh_nodes": len(tree), "build_s": round(build_s, 2),
               "time_no_bvh_s": t_no, "time_bvh_s": t_bvh, "wall_no_bvh_s": w_no, "wall_bvh_s": w_bvh,
               "hits_no_bvh": int(hit_a.sum()), "hits_bvh": int(hits_b["hit"].sum()),
               "sphere_tests_per_s_G": round(n * a.rays / t_no / 1e9, 1),
               "check_rays_no_bvh": ka, "check_rays_bvh": k, "bvh_check": bvh_check,
               "any_hit_equals_oracle": ok_a, "bvh_hits_equal_oracle": ok_b}
        if pub:
            row["published_s"] = list(pub)
            row["published_over_gpu"] = [round(pub[0] / t_no, 1), round(pub[1] / t_bvh, 1)]
        rows.append(row)
        print(json.dumps(row), flush=True)
        del pre, spheres, tree
    n = [x["spheres"] for x in rows]
    out = {"source": "scripts/bench_mode_published.py", "seed": a.seed, "rays_per_loop": a.rays,
           "note": "GPU times are device times (HIP events) of one batch launch per loop over the same rays the "
                   "reference's loops draw; the published times are the reference's clock() seconds on its "
                   "authors' CPU with an unrecorded ray count (results/benchmark_data.txt), so the ratios compare "
                   "rows, not equal work",
           "points": rows,
           "loglog_slope_gpu": {"no_bvh": round(slope(n, [x["time_no_bvh_s"] for x in rows]), 3),
                                "bvh": round(slope(n, [x["time_bvh_s"] for x in rows]), 3)},
           "loglog_slope_published": {"no_bvh": round(slope(list(PUBLISHED), [v[0] for v in PUBLISHED.values()]), 3),
                                      "bvh": round(slope(list(PUBLISHED), [v[1] for v in PUBLISHED.values()]), 3)}}
    with open(a.out + ".json", "w") as f:
        json.dump(out, f, indent=1)
    with open(a.out + "_benchmark_data.txt", "w") as f:
        for x in rows:
            f.write(f"{x['spheres']} {x['time_no_bvh_s']:f} {x['time_bvh_s']:f}\n")
    print(json.dumps({k: v for k, v in out.items() if k != "points"}))
    r.close()
    ok = all(x["any_hit_equals_oracle"] and x["bvh_hits_equal_oracle"] for x in rows)
    return 0 if ok else 3


if __name__ == "__main__":
    sys.exit(main())
