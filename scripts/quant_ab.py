"""A/B of a bounce-walk node option (default MIRT_OPT_QUANT: 64-B fp16
HNodes vs 48-B 8-bit QNodes; --opt HNODE_DFS: breadth- vs depth-first HNode
numbering), one context, serial launches on one stream.

Prints per setting: primary / bounce pass ms (HIP events the library records
around them), the bounce-level node/sphere tests (mirt_count_frame) and the
frame's SHA-256, which must agree between the settings.
usage: python scripts/quant_ab.py [--workload 1080p_10k] [--reps 20] [--opt QUANT]
"""
import argparse
import hashlib
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (one HIP runtime: torch's, as in bench.py)

mirt = importlib.import_module("cs201_sah-bvh_ray_tracer_amd")
WORKLOADS = {
    "1080p_10k": (1920, 1080, "render", 10000),
    "1080p_100k": (1920, 1080, "render", 100000),
    "4k_10k": (3840, 2160, "render", 10000),
    "4k_1m": (3840, 2160, "bench", 1000000),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="1080p_10k")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--opt", default="QUANT", choices=["QUANT", "HNODE_DFS"])
    a = ap.parse_args()
    W, H, kind, n = WORKLOADS[a.workload]
    s = mirt.create_random_spheres(n, 1) if kind == "render" else mirt.create_benchmark_spheres(n, 1)
    b = mirt.build_bvh(s)
    cam = mirt.default_camera()
    out = {}
    with mirt.Renderer(0) as r:
        r.upload(s, b)
        for q in (0, 1, 0, 1):
            r.set_option(getattr(mirt.abi, "OPT_" + a.opt), q)
            img = r.render_frame(cam, W, H, depth=5, seed=1)
            ph = []
            for _ in range(a.reps):
                r.render_frame(cam, W, H, depth=5, seed=1)
                ph.append(r.last_phase_ms())
            c = r.count_frame(cam, W, H, depth=5, seed=1)
            p = np.array(ph)
            out[f"quant{q}"] = {
                "primary_ms": round(float(np.median(p[:, 0])), 4),
                "bounce_ms": round(float(np.median(p[:, 1])), 4),
                "bounce_min_ms": round(float(p[:, 1].min()), 4),
                "nodes_bounce": int(c["nodes"] - c["nodes_primary"]),
                "spheres_bounce": int(c["spheres"] - c["spheres_primary"]),
                "sha": hashlib.sha256(np.ascontiguousarray(img).tobytes()).hexdigest()[:16],
            }
            print(a.workload, f"{a.opt}={q}", json.dumps(out[f"quant{q}"]), flush=True)
    assert out["quant0"]["sha"] == out["quant1"]["sha"], "node formats disagree"


if __name__ == "__main__":
    main()
