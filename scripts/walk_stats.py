"""Per-walk work and time at one depth: node tests, sphere tests and wave
steps (lane_steps / 64) of the instrumented kernel, and the frame time of
the timed kernel, for each (prune, ordered) setting.

    python scripts/walk_stats.py [--depth 1] [--spheres 10000]
"""
import argparse
import importlib
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mirt = importlib.import_module("cs201_sah-bvh_ray_tracer_amd")
abi = mirt.abi


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--depth", type=int, default=1)
    ap.add_argument("--spheres", type=int, default=10000)
    a = ap.parse_args()
    s = mirt.create_random_spheres(a.spheres, 1)
    b = mirt.build_bvh(s)
    r = mirt.Renderer(0)
    r.upload(s, b)
    cam = mirt.default_camera()
    for prune, ordered in [(0, 0), (1, 0), (1, 1)]:
        r.set_option(abi.OPT_PRUNE, prune)
        r.set_option(abi.OPT_ORDERED, ordered)
        c = r.count_frame(cam, 1920, 1080, depth=a.depth, seed=1)
        ts = []
        for _ in range(6):
            r.render_frame(cam, 1920, 1080, depth=a.depth, seed=1)
            ts.append(r.last_kernel_ms)
        print(json.dumps({"prune": prune, "ordered": ordered, "depth": a.depth, "ms": round(float(np.median(ts[1:])), 3),
                          "nodes_per_ray": round(c["nodes"] / c["rays"], 1),
                          "spheres_per_ray": round(c["spheres"] / c["rays"], 1),
                          "wave_steps": c["lane_steps"] // 64, "rays": c["rays"]}), flush=True)
    r.close()


if __name__ == "__main__":
    main()
