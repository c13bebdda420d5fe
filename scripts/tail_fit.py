"""Is the bounce pass throughput- or tail-bound? Time both passes at several
frame heights (same scene/camera) and fit t = a * H + b: b is the part of a
launch that does not shrink with the work (drain / tail).

    python scripts/tail_fit.py
"""
import importlib
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mirt = importlib.import_module("cs201_sah-bvh_ray_tracer_amd")


def main():
    s = mirt.create_random_spheres(10000, 1)
    b = mirt.build_bvh(s)
    r = mirt.Renderer(0)
    r.upload(s, b)
    cam = mirt.default_camera()
    rows = []
    for H in (135, 270, 540, 1080, 2160):
        ph = []
        for i in range(6):
            r.render_frame(cam, 1920, H, depth=5, seed=1)
            ph.append(r.last_phase_ms())
        p = np.median(np.array(ph[1:]), axis=0)
        rows.append((H, p[0], p[1]))
        print(json.dumps({"H": H, "primary_ms": round(float(p[0]), 4), "bounce_ms": round(float(p[1]), 4)}), flush=True)
    a = np.array(rows)
    for k, name in ((1, "primary"), (2, "bounce")):
        slope, icpt = np.polyfit(a[:, 0], a[:, k], 1)
        print(json.dumps({"pass": name, "ms_per_1080_rows": round(float(slope * 1080), 4),
                          "fixed_ms": round(float(icpt), 4)}))
    r.close()


if __name__ == "__main__":
    main()
