"""Per-shard kernel time of the default frame on ONE GPU, for the row-block
sharding the multi-GPU bench uses: rendering shard k of N on one device is
exactly rank k's launch at N GPUs, so max over k predicts the per-GPU part
of an N-GPU step (the RCCL gather comes on top).

    python scripts/shard_times.py [--reps 10] [--weak]

--weak: the bench's default step -- at N GPUs every rank renders its rows
of N frames in one launch (accumulated), so the per-rank work stays one
frame's worth.

--pipeline P: time the bench's timed loop instead of single launches -- P
contexts take successive steps of shard k on their own streams, with
--blocks persistent bounce workgroups per launch (the bench's defaults: 4 and
1.5 per CU) -- and report each shard's per-rank Mrays/s (the RCCL gather
comes on top).
"""
import argparse
import importlib
import json
import os
import sys
import time

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
    ap.add_argument("--pipeline", type=int, default=0, help="time P contexts in flight (bench loop)")
    ap.add_argument("--blocks", type=int, default=-1, help="bounce workgroups with --pipeline (-1: 1.5 per CU)")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--scene", choices=("render", "bench"), default="render",
                    help="create_random_sphere scene (main.c) or benchmark spheres (benchmark.c:307-314)")
    ap.add_argument("--spp", type=int, default=1, help="jittered samples per frame (BASELINE configs[4]: 4)")
    ap.add_argument("--batch", type=int, default=1,
                    help="with --pipeline: consecutive frames per launch (each frame's display its own slab)")
    ap.add_argument("--tail-grid", type=int, default=0,
                    help="with --pipeline: the last N launches of each timed burst run their bounce pass on the "
                         "full persistent grid (bench.py --tail-grid)")
    ap.add_argument("--copy", action="store_true",
                    help="with --pipeline: after every step a slab-sized D2D copy on one more stream, waiting "
                         "for that step's frame (prices the RCCL gather's stream against the hardware queues)")
    a = ap.parse_args()
    if a.pipeline:
        return pipelined(a)
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


def pipelined(a):
    W, H = a.width, a.height
    s = (mirt.create_random_spheres(a.spheres, 1) if a.scene == "render"
         else mirt.create_benchmark_spheres(a.spheres, 1))
    b = mirt.build_bvh(s)
    blocks = a.blocks if a.blocks >= 0 else 3 * torch.cuda.get_device_properties(0).multi_processor_count // 2
    rs = [mirt.Renderer(0) for _ in range(a.pipeline)]
    for r in rs:
        r.upload(s, b)
        r.set_option(mirt.abi.OPT_BOUNCE_BLOCKS, blocks)
        for ov in a.opt:
            o, v = (int(x) for x in ov.split("="))
            r.set_option(o, v)
    streams = [torch.cuda.ExternalStream(r.stream_handle) for r in rs]
    cam = mirt.default_camera()
    for world in (int(w) for w in a.worlds.split(",")):
        rows = shard.slab_rows(H, 8, world)
        frames = a.spp * (world if a.weak else 1) * a.batch
        slabs = [torch.zeros((frames, rows, W), dtype=torch.int32, device="cuda") for _ in rs]
        cstream = torch.cuda.Stream() if a.copy else None
        dst = torch.zeros((rows, W), dtype=torch.int32, device="cuda") if a.copy else None
        # an accumulation buffer folds the samples of a jittered frame / the
        # frames of the weak step; batched fresh frames stay raw slabs
        accs = [torch.zeros((rows, W, 3), dtype=torch.float32, device="cuda") if (a.spp > 1 or a.weak) else None
                for _ in rs]
        per = []
        for k in range(world):
            fd = mirt.frame_desc(W, H, a.depth, True, 1, 0, False, 1, 8, k, world, frames, a.spp > 1)

            def run(n):
                for i in range(n):
                    j = i % len(rs)
                    tail = i >= n - a.tail_grid
                    if tail:
                        rs[j].set_option(mirt.abi.OPT_BOUNCE_BLOCKS, 0)
                    rs[j].render_frame_device(cam, fd, slabs[j].data_ptr(),
                                              accs[j].data_ptr() if accs[j] is not None else None,
                                              streams[j].cuda_stream)
                    if tail:
                        rs[j].set_option(mirt.abi.OPT_BOUNCE_BLOCKS, blocks)
                    if cstream is not None:
                        cstream.wait_stream(streams[j])
                        with torch.cuda.stream(cstream):
                            dst.copy_(slabs[j][0])
            run(2 * len(rs))
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run(a.steps)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            per.append(W * H * frames / world * a.steps / el / 1e6)
        print(json.dumps({"spheres": a.spheres, "scene": a.scene, "size": [W, H], "spp": a.spp, "copy": a.copy,
                          "batch": a.batch, "tail_grid": a.tail_grid,
                          "world": world, "frames": frames, "pipeline": a.pipeline,
                          "blocks": blocks, "per_rank_mrays_s": [round(p, 1) for p in per],
                          "min_per_rank_mrays_s": round(min(per), 1),
                          "pred_job_mrays_s_no_gather": round(min(per) * world, 1)}), flush=True)
    for r in rs:
        r.close()


if __name__ == "__main__":
    main()
