"""Per-shard kernel time of the default frame on ONE GPU, for the row-block
sharding the multi-GPU bench uses: rendering shard k of N on one device is
exactly rank k's launch at N GPUs, so max over k predicts the per-GPU part
of an N-GPU step (the RCCL gather comes on top).

    python scripts/shard_times.py [--reps 10] [--weak]

--weak: the bench's default step -- at N GPUs every rank renders its rows
of N frames in one launch (accumulated), so the per-rank work stays one
frame's worth.
"""
import argparse
import importlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
mirt = importlib.import_module("cs201_sah-bvh_ray_tracer_amd")
shard = importlib.import_module("cs201_sah-bvh_ray_tracer_amd.shard")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spheres", type=int, default=10000)
    ap.add_argument("--depth", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--weak", action="store_true", help="N frames in flight at N shards (the bench default)")
    ap.add_argument("--opt", action="append", default=[], help="option=value (mirt_set_option), repeatable")
    a = ap.parse_args()
    W, H = a.width, a.height
    s = mirt.create_random_spheres(a.spheres, 1)
    b = mirt.build_bvh(s)
    r = mirt.Renderer(0)
    r.upload(s, b)
    for ov in a.opt:
        o, v = (int(x) for x in ov.split("="))
        r.set_option(o, v)
    cam = mirt.default_camera()
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    for world in (int(w) for w in a.worlds.split(",")):
        rows = shard.slab_rows(H, 8, world)
        frames = world if a.weak else 1
        slab = torch.zeros((frames, rows, W), dtype=torch.int32, device="cuda")
        acc = torch.zeros((rows, W, 3), dtype=torch.float32, device="cuda") if frames > 1 else None
        accp = acc.data_ptr() if acc is not None else None
        per = []
        phases = []
        for k in range(world):
            fd = mirt.frame_desc(W, H, a.depth, True, 1, 0, False, 1, 8, k, world, frames)
            for _ in range(3):
                r.render_frame_device(cam, fd, slab.data_ptr(), accp, stream.cuda_stream)
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.reps)]
            for e0, e1 in ev:
                e0.record(stream)
                r.render_frame_device(cam, fd, slab.data_ptr(), accp, stream.cuda_stream)
                e1.record(stream)
            torch.cuda.synchronize()
            per.append(float(np.median([e0.elapsed_time(e1) for e0, e1 in ev])))
            r.render_frame_device(cam, fd, slab.data_ptr(), accp, stream.cuda_stream)
            phases.append([round(float(v), 4) for v in r.last_phase_ms()])
        print(json.dumps({"opts": a.opt, "spheres": a.spheres, "world": world, "max_ms": round(max(per), 4), "mean_ms": round(float(np.mean(per)), 4),
                          "per_shard_ms": [round(p, 4) for p in per], "phases_ms": phases,
                          "frames": frames,
                          "pred_mrays_s_no_gather": round(W * H * frames / max(per) / 1e3, 1)}), flush=True)
    r.close()


if __name__ == "__main__":
    main()
