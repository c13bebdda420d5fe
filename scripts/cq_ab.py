"""The continuation queue (MIRT_OPT_CONT_QUEUE) on the frame that runs alone:
the blocking call into page-locked memory (median of --calls) and its two
passes' HIP-event times, queue off / on, per scene; every frame must equal
the queue-off frame (and, at 10k, the reference's golden).

    python scripts/cq_ab.py [--spheres 10000,100000] [--rounds 3]
"""
import argparse
import ctypes
import hashlib
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
m = importlib.import_module("cs201_sah-bvh_ray_tracer_amd")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spheres", default="10000,100000")
    ap.add_argument("--calls", type=int, default=21)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    a = ap.parse_args()
    W, H = a.width, a.height
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))["frames"]
    for n in (int(x) for x in a.spheres.split(",")):
        s = m.create_random_spheres(n, 1)
        b = m.build_bvh(s)
        r = m.Renderer(0)
        r.upload(s, b)
        cam = m.default_camera()
        hb = m.HostBuffer((H, W, 4))
        r.set_option(m.abi.OPT_CONT_QUEUE, 0)
        ref = r.render_frame(cam, W, H, depth=5, seed=1)
        res = {}
        for rnd in range(a.rounds):
            for cq in (0, 1):
                r.set_option(m.abi.OPT_CONT_QUEUE, cq)
                r.render_frame_into(cam, W, H, hb.array, depth=5, seed=1)
                same = bool((hb.array == ref).all())
                dts, ph = [], []
                for _ in range(a.calls):
                    t0 = time.perf_counter()
                    r.render_frame_into(cam, W, H, hb.array, depth=5, seed=1)
                    dts.append(time.perf_counter() - t0)
                    ph.append(r.last_phase_ms())
                    same = same and bool((hb.array == ref).all())
                ms = sorted(dts)[len(dts) // 2] * 1e3
                st = np.zeros(5, np.uint32)
                k = m.load().mirt_cont_queue_stats(r.h, st.ctypes.data_as(ctypes.c_void_p), 5)
                ph.sort(key=lambda p: p[1])
                res.setdefault(cq, []).append(ms)
                print(json.dumps({"spheres": n, "round": rnd, "cont_queue": cq, "blocking_ms": round(ms, 4),
                                  "primary_ms": round(ph[len(ph) // 2][0], 4), "bounce_ms": round(ph[len(ph) // 2][1], 4),
                                  "equal_to_queue_off": same,
                                  "cq_stats": st[:max(k, 0)].tolist() if cq else None}), flush=True)
        key = f"{W}x{H}_render{n}_d5_m1_b1_s1_c0_step1"
        g = gold.get(key, {}).get("sha")
        print(json.dumps({"spheres": n, "best_ms": {k: round(min(v), 4) for k, v in res.items()},
                          "golden": None if g is None else hashlib.sha256(ref.tobytes()).hexdigest() == g}), flush=True)
        hb.close()
        r.close()


if __name__ == "__main__":
    main()
