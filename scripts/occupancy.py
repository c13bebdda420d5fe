"""Does the frame kernel scale with work (throughput-bound) or is it set by
its slowest tiles (tail-bound)? Times 1080p/10k frames for several
workgroup sizes and for 1/1, 1/8 and 1/32 of the rows (row-block shards).

    python scripts/occupancy.py
"""
import importlib
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mirt = importlib.import_module("cs201_sah-bvh_ray_tracer_amd")
abi = mirt.abi


def main():
    s = mirt.create_random_spheres(10000, 1)
    b = mirt.build_bvh(s)
    r = mirt.Renderer(0)
    r.upload(s, b)
    cam = mirt.default_camera()
    for depth, trav in [(1, abi.TRAV_TILE), (5, abi.TRAV_TILE)]:
        r.set_option(abi.OPT_TRAVERSAL, trav)
        for bw in (1, 2, 4, 8):
            r.set_option(abi.OPT_BLOCK_WAVES, bw)
            for shards in (1, 8, 32):
                ts = []
                for _ in range(4):
                    r.render_frame(cam, 1920, 1080, depth=depth, num_shards=shards)
                    ts.append(r.last_kernel_ms)
                t = float(np.median(ts[1:]))
                print(json.dumps({"depth": depth, "trav": trav, "block_waves": bw, "fraction": f"1/{shards}",
                                  "ms": round(t, 3), "ms_x_shards": round(t * shards, 2)}), flush=True)
    r.close()


if __name__ == "__main__":
    main()
