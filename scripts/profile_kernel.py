"""Render frames of one schedule for counter profiling, and print the
reference-DFS work and SIMD efficiency of every schedule.

    python scripts/profile_kernel.py --counts                 # work + efficiency table
    python scripts/profile_kernel.py --trav 1 --fast 1 --depth 5 --frames 5 [--opt 7=0]  # frames to profile
"""
import argparse
import importlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mirt = importlib.import_module("cs201_sah-bvh_ray_tracer_amd")
abi = mirt.abi


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="render10000")
    ap.add_argument("--W", type=int, default=1920)
    ap.add_argument("--H", type=int, default=1080)
    ap.add_argument("--trav", type=int, default=abi.TRAV_WAVEFRONT)
    ap.add_argument("--fast", type=int, default=1)
    ap.add_argument("--depth", type=int, default=5)
    ap.add_argument("--frames", type=int, default=3)
    ap.add_argument("--counts", action="store_true")
    ap.add_argument("--opt", action="append", default=[], help="OPTION=VALUE (mirt_set_option), repeatable")
    a = ap.parse_args()
    kind = "render" if a.scene.startswith("render") else "bench"
    n = int(a.scene[len(kind):])
    s = mirt.create_random_spheres(n, 1) if kind == "render" else mirt.create_benchmark_spheres(n, 1)
    b = mirt.build_bvh(s)
    r = mirt.Renderer(0)
    r.upload(s, b)
    cam = mirt.default_camera()
    if a.counts:
        for depth in (1, 5):
            for trav in (abi.TRAV_TILE,):
                r.set_option(abi.OPT_TRAVERSAL, trav)
                c = r.count_frame(cam, a.W, a.H, depth=depth)
                c.update(scene=a.scene, depth=depth, trav=trav,
                         simd_eff=round(c["nodes"] / max(c["lane_steps"], 1), 4),
                         nodes_per_ray=round(c["nodes"] / max(c["rays"], 1), 1),
                         spheres_per_ray=round(c["spheres"] / max(c["rays"], 1), 1))
                print(json.dumps(c), flush=True)
        return
    r.set_option(abi.OPT_TRAVERSAL, a.trav)
    r.set_option(abi.OPT_FAST_SLAB, a.fast)
    for kv in a.opt:
        k, v = kv.split("=")
        r.set_option(int(k), int(v))
    for _ in range(a.frames):
        r.render_frame(cam, a.W, a.H, depth=a.depth)
        print(json.dumps({"trav": a.trav, "fast": a.fast, "depth": a.depth, "kernel_ms": round(r.last_kernel_ms, 3)}))
    r.close()


if __name__ == "__main__":
    main()
