"""Where does the bounce kernel's time go? Steady state vs the drain after the
bounce queue runs dry, lanes per loop iteration, longest walks and chains
(mirt_bounce_stats).

    python scripts/bounce_stats.py [--threshold 20] [--spheres 10000]
"""
import argparse
import importlib
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mirt = importlib.import_module("cs201_sah-bvh_ray_tracer_amd")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spheres", type=int, default=10000)
    ap.add_argument("--threshold", type=int, default=20)
    ap.add_argument("--dump", default=None, help="save the raw per-wave records (.npy)")
    ap.add_argument("--shards", default="1", help="comma list: shard 0 of N for each N")
    a = ap.parse_args()
    s = mirt.create_random_spheres(a.spheres, 1)
    b = mirt.build_bvh(s)
    r = mirt.Renderer(0)
    r.upload(s, b)
    r.set_option(mirt.abi.OPT_BOUNCE_THRESHOLD, a.threshold)
    cam = mirt.default_camera()
    for ns in [int(v) for v in a.shards.split(",")]:
        report(r, cam, ns, a)
    r.close()


def report(r, cam, ns, a):
    r.bounce_stats(cam, 1920, 1080, shard=0, num_shards=ns)
    d = r.bounce_stats(cam, 1920, 1080, shard=0, num_shards=ns).astype(np.float64)
    if a.dump:
        np.save(a.dump + f".{ns}.npy", d)
    t0 = d[:, 4].min()
    end = (d[:, 6] - t0) / 100.0
    dry = d[:, 5][d[:, 5] > 0]
    walk = (d[:, 7].astype(np.uint64) & np.uint64(0xffffffff)).astype(np.int64)
    chain = (d[:, 7].astype(np.uint64) >> np.uint64(32)).astype(np.int64)
    tq = d[:, 9][d[:, 9] > 0]
    print(json.dumps({
        "shards": ns,
        "waves": len(d), "span_us": round(float(end.max()), 1),
        "quad_drain_waves": int(len(tq)),
        "quad_drain_start_us_p50": round(float(np.median(tq - t0) / 100.0), 1) if len(tq) else None,
        "quad_drain_iters_max": int(d[:, 8].max()), "quad_drain_iters_p50": int(np.median(d[:, 8][d[:, 8] > 0]))
        if (d[:, 8] > 0).any() else 0,
        "queue_dry_us_median": round(float(np.median(dry - t0) / 100.0), 1),
        "wave_end_us_p50": round(float(np.median(end)), 1), "wave_end_us_p90": round(float(np.percentile(end, 90)), 1),
        "lanes_per_iter": round(float(d[:, 1].sum() / d[:, 0].sum()), 2),
        "lanes_per_iter_before_dry": round(float((d[:, 1] - d[:, 3]).sum() / (d[:, 0] - d[:, 2]).sum()), 2),
        "lanes_per_iter_after_dry": round(float(d[:, 3].sum() / max(1.0, d[:, 2].sum())), 2),
        "iters_after_dry_frac": round(float(d[:, 2].sum() / d[:, 0].sum()), 3),
        "lane_steps": int(d[:, 1].sum()),
        "fallback_lane_steps": int(d[:, 10].sum()), "fallbacks": int(d[:, 11].sum()),
        "fallback_share_of_lane_steps": round(float(d[:, 10].sum() / max(1.0, d[:, 1].sum())), 4),
        "longest_walk_p50": int(np.median(walk)), "longest_walk_max": int(walk.max()),
        "longest_chain_p50": int(np.median(chain)), "longest_chain_max": int(chain.max())}), flush=True)


if __name__ == "__main__":
    main()
