"""One blocking frame split into n row-block shards rendered concurrently on
ONE GPU (mirt_multi copy mode: n ctxs, n streams, the slabs copied to the
first ctx and de-interleaved there, one D2H), against the single-ctx blocking
frame: does overlapping the shards' primary passes with each other's bounce
drain shorten a lone frame? 1080p / 10k depth 5, median of 21 enqueue+wait.

    python scripts/split_frame.py [--shards 1,2,4,8] [--blocks 0,320]
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
m = importlib.import_module("cs201_sah-bvh_ray_tracer_amd")


def med(fn, calls=21):
    fn()
    dts = []
    for _ in range(calls):
        t0 = time.perf_counter()
        fn()
        dts.append(time.perf_counter() - t0)
    return sorted(dts)[len(dts) // 2] * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shards", default="1,2,3,4,8")
    ap.add_argument("--blocks", default="0", help="bounce workgroups per shard ctx (0: the full grid)")
    a = ap.parse_args()
    W, H = 1920, 1080
    s = m.create_random_spheres(10000, 1)
    b = m.build_bvh(s)
    cam = m.default_camera()
    r = m.Renderer(0)
    r.upload(s, b)
    ref = r.render_frame(cam, W, H, depth=5, seed=1)
    hb = m.HostBuffer((H, W, 4))
    out = {"single_pinned_ms": round(med(lambda: r.render_frame_into(cam, W, H, hb.array, depth=5, seed=1)), 4)}
    r.close()
    fd = m.frame_desc(W, H, depth=5, seed=1)
    ok = True
    for n in [int(v) for v in a.shards.split(",")]:
        mr = m.MultiRenderer([0] * n, copy=True)
        mr.upload(s, b)
        for bb in [int(v) for v in a.blocks.split(",")]:
            mr.set_option(m.abi.OPT_BOUNCE_BLOCKS, bb)

            def frame():
                mr.render_frame_async(cam, fd, hb)
                mr.wait()
            hb.array[:] = 0
            out[f"split{n}_b{bb}_ms"] = round(med(frame), 4)
            ok = ok and bool((hb.array == ref).all())
        mr.close()
    out["frames_equal"] = ok
    print(json.dumps(out), flush=True)
    hb.close()


if __name__ == "__main__":
    main()
