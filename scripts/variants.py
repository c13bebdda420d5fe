"""A/B the kernel schedules in ONE process (interleaved rounds), checking
that every variant produces the same bytes. Prints one JSON line per
(scene, depth, variant) with median / min kernel ms.

    python scripts/variants.py [--rounds 5] [--scenes render10000,render100000]
"""
import argparse
import hashlib
import importlib
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mirt = importlib.import_module("cs201_sah-bvh_ray_tracer_amd")
abi = mirt.abi

VARIANTS = {
    "uniform_exact": (abi.TRAV_UNIFORM, 0), "uniform_fast": (abi.TRAV_UNIFORM, 1),
    "lane_exact": (abi.TRAV_LANE, 0), "lane_fast": (abi.TRAV_LANE, 1),
    "hybrid_exact": (abi.TRAV_HYBRID, 0), "hybrid_fast": (abi.TRAV_HYBRID, 1),
    "lanenp_fast": (abi.TRAV_LANE_NP, 1), "hybridnp_fast": (abi.TRAV_HYBRID_NP, 1),
    "wavefront_fast": (abi.TRAV_WAVEFRONT, 1), "wavefront_exact": (abi.TRAV_WAVEFRONT, 0),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--scenes", default="render10000,render100000")
    ap.add_argument("--depths", default="1,5")
    ap.add_argument("--variants", default=",".join(VARIANTS))
    ap.add_argument("--W", type=int, default=1920)
    ap.add_argument("--H", type=int, default=1080)
    args = ap.parse_args()
    r = mirt.Renderer(0)
    cam = mirt.default_camera()
    names = args.variants.split(",")
    for scene in args.scenes.split(","):
        kind = "render" if scene.startswith("render") else "bench"
        n = int(scene[len(kind):])
        s = mirt.create_random_spheres(n, 1) if kind == "render" else mirt.create_benchmark_spheres(n, 1)
        b = mirt.build_bvh(s)
        r.upload(s, b)
        for depth in map(int, args.depths.split(",")):
            times = {v: [] for v in names}
            shas = {}
            for rnd in range(args.rounds + 1):
                for v in names:
                    trav, fast = VARIANTS[v]
                    r.set_option(abi.OPT_TRAVERSAL, trav)
                    r.set_option(abi.OPT_FAST_SLAB, fast)
                    img = r.render_frame(cam, args.W, args.H, depth=depth, seed=1)
                    if rnd == 0:
                        shas[v] = hashlib.sha256(img.tobytes()).hexdigest()
                    else:
                        times[v].append(r.last_kernel_ms)
            same = len(set(shas.values())) == 1
            for v in names:
                t = np.array(times[v])
                print(json.dumps({"scene": scene, "depth": depth, "variant": v, "median_ms": round(float(np.median(t)), 3),
                                  "min_ms": round(float(t.min()), 3),
                                  "mrays_s": round(args.W * args.H / np.median(t) / 1e3, 2),
                                  "all_variants_identical": same, "sha": shas[v][:16]}), flush=True)
    r.close()


if __name__ == "__main__":
    main()
