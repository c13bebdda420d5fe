"""Per-wave timing of the frame kernel (diagnostic): is a frame set by
throughput or by its slowest 8x8 tiles? Saves the raw table to
gpurun_out/wave_stats_<depth>.npy and prints a summary.

    python scripts/wave_stats.py [depth,trav,ordered ...]
"""
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
mirt = importlib.import_module("cs201_sah-bvh_ray_tracer_amd")
abi = mirt.abi


def summarize(st, W, H, label):
    tiles_x = (W + 7) // 8
    t0 = st[:, 2].astype(np.int64)
    t1 = st[:, 3].astype(np.int64)
    base = t0.min()
    t0 -= base
    t1 -= base
    dur = (t1 - t0) / 100.0          # us (100 MHz clock)
    span = t1.max() / 100.0
    steps = st[:, 1] / 64.0          # every lane counts each step
    # concurrency: average number of live waves over the span
    conc = dur.sum() / span
    # time at which 90% / 99% of waves had finished
    ends = np.sort(t1) / 100.0
    out = {"label": label, "waves": int(len(st)), "span_us": round(span, 1),
           "avg_live_waves": round(float(conc), 1),
           "dur_us_p50": round(float(np.percentile(dur, 50)), 1), "dur_us_p90": round(float(np.percentile(dur, 90)), 1),
           "dur_us_p99": round(float(np.percentile(dur, 99)), 1), "dur_us_max": round(float(dur.max()), 1),
           "steps_p50": float(np.percentile(steps, 50)), "steps_p99": float(np.percentile(steps, 99)),
           "steps_max": float(steps.max()),
           "us_per_step_median": round(float(np.median(dur / np.maximum(steps, 1))), 3),
           "t_90pct_done_us": round(float(ends[int(0.9 * len(ends))]), 1),
           "t_99pct_done_us": round(float(ends[int(0.99 * len(ends))]), 1),
           "start_us_max": round(float(t0.max() / 100.0), 1)}
    slow = np.argsort(-dur)[:8]
    out["slowest"] = [{"tile_x": int(st[i, 0] % tiles_x), "tile_y": int(st[i, 0] // tiles_x), "us": round(float(dur[i]), 1),
                       "steps": float(steps[i]), "start_us": round(float(t0[i] / 100.0), 1)} for i in slow]
    print(json.dumps(out), flush=True)


def main():
    s = mirt.create_random_spheres(10000, 1)
    b = mirt.build_bvh(s)
    r = mirt.Renderer(0)
    r.upload(s, b)
    cam = mirt.default_camera()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    configs = [(1, abi.TRAV_TILE, 0), (1, abi.TRAV_TILE, 1)]
    if len(sys.argv) > 1:   # depth,trav,ordered ...
        configs = [tuple(int(v) for v in a.split(",")) for a in sys.argv[1:]]
    for depth, trav, ordered in configs:
        r.set_option(abi.OPT_TRAVERSAL, trav)
        r.set_option(abi.OPT_ORDERED, ordered)
        r.wave_stats(cam, 1920, 1080, depth=depth)           # warm
        st = r.wave_stats(cam, 1920, 1080, depth=depth)
        np.save(os.path.join(ROOT, "gpurun_out", f"wave_stats_d{depth}_t{trav}_o{ordered}.npy"), st)
        summarize(st, 1920, 1080, f"1080p 10k depth {depth} trav {trav} ordered {ordered}")
    r.close()


if __name__ == "__main__":
    main()
