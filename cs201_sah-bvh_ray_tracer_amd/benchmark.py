"""The reference's benchmark mode on the GPU: run_benchmark_with_plotting
(benchmark.c:283-332) with its two timed loops as batched HIP launches.

Per sweep point, on ONE glibc rand() stream exactly as the reference
consumes it (srand once, benchmark.c:286 -- a fixed seed here instead of
time(NULL)):
  spheres      n x create_benchmark_sphere at uniform centres in
               [-world/2, world/2)^3 (benchmark.c:307-314)
  tree         build_bvh_node(spheres, 0, n - 1, 20) (benchmark.c:317: the
               last sphere stays out of the tree, as in the reference)
  no-BVH loop  num_rays rays (benchmark.c:176-185), each tested against every
               sphere; counts the rays with some hit (benchmark.c:190-205)
               -> Renderer.any_hit(rays, use_bvh=False): one launch, the
               sphere loop split into chunks across the chip
  BVH loop     num_rays fresh rays, ray_bvh_intersect each (benchmark.c:
               224-255) -> Renderer.closest_hit(rays, use_bvh=True)
and save_benchmark_data's line "n time_no_bvh time_with_bvh" (seconds,
benchmark.c:160-170). Times are device times of the launches (HIP events),
median over `reps` repetitions; the PCIe-inclusive wall time of each call is
reported beside them.
"""
import time

import numpy as np

from .renderer import RandState, build_bvh, create_bench_rays, create_benchmark_spheres

DEFAULT_COUNTS = list(range(5000, 50001, 5000))   # benchmark.c:288-296
NUM_RAYS = 10000                                   # benchmark.c:298
WORLD_SIZE = 1000.0                                # benchmark.c:299


def sweep(counts=DEFAULT_COUNTS, num_rays=NUM_RAYS, seed=1, world_size=WORLD_SIZE):
    """The sweep's inputs in the reference's draw order: yields (n, spheres
    after the in-place build, tree, no-BVH rays, BVH rays)."""
    st = RandState(seed)
    for n in counts:
        spheres = create_benchmark_spheres(n, world_size=world_size, state=st)
        tree = build_bvh(spheres, 0, n - 1, 20)
        rays_a = create_bench_rays(num_rays, st)
        rays_b = create_bench_rays(num_rays, st)
        yield n, spheres, tree, rays_a, rays_b


def _timed(fn, renderer, reps):
    out, dev, wall = None, [], []
    for _ in range(max(1, reps)):
        t0 = time.perf_counter()
        out = fn()
        wall.append(time.perf_counter() - t0)
        dev.append(renderer.last_kernel_ms / 1e3)
    return out, float(np.median(dev)), float(np.median(wall))


def run_benchmark(renderer, counts=DEFAULT_COUNTS, num_rays=NUM_RAYS, seed=1, world_size=WORLD_SIZE, reps=5,
                  data_path=None, verbose=False):
    """Returns one dict per sweep point; appends save_benchmark_data lines
    to data_path if given (the reference removes the file first,
    benchmark.c:285)."""
    rows = []
    for n, spheres, tree, rays_a, rays_b in sweep(counts, num_rays, seed, world_size):
        renderer.upload(spheres, tree)
        hit_a, t_no, w_no = _timed(lambda: renderer.any_hit(rays_a, use_bvh=False), renderer, reps)
        hits_b, t_bvh, w_bvh = _timed(lambda: renderer.closest_hit(rays_b, use_bvh=True), renderer, reps)
        _, t_closest, _ = _timed(lambda: renderer.closest_hit(rays_a, use_bvh=False), renderer, reps)
        row = {"spheres": n, "rays": num_rays, "tests": n * num_rays, "bvh_nodes": len(tree),
               "hits_no_bvh": int(hit_a.sum()), "hits_bvh": int(hits_b["hit"].sum()),
               "time_no_bvh_s": t_no, "time_bvh_s": t_bvh, "time_no_bvh_closest_s": t_closest,
               "wall_no_bvh_s": w_no, "wall_bvh_s": w_bvh,
               "hit_no_bvh": hit_a, "hit_bvh": hits_b["hit"].astype(np.int32)}
        rows.append(row)
        if verbose:  # benchmark.c:207-216, 245-250
            print(f"Testing with {n} spheres:\nNo BVH:\nTime: {t_no:f} seconds\nIntersection tests: {n * num_rays}\n"
                  f"Intersections found: {row['hits_no_bvh']}\n\nWith BVH:\nTime: {t_bvh:f} seconds\n"
                  f"Intersections found: {row['hits_bvh']}\n\n----------------------------------------", flush=True)
        if data_path:
            with open(data_path, "a") as f:
                f.write(f"{n} {t_no:f} {t_bvh:f}\n")
    return rows
