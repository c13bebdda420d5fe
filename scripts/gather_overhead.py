"""Host cost of the N > 1 bench launch (render_local + the RCCL gather of every
frame + the de-interleave), measured on one GPU with a world-1 nccl group:
at N = 8 a rank's launch of 4 frames is ~0.5 ms of GPU work, so the host must
enqueue a launch and its gather in less than that or the rank becomes
host-bound. Prints the host milliseconds per launch (enqueue only, no sync)
and the GPU milliseconds per launch of the same loop.

    MASTER_ADDR=127.0.0.1 MASTER_PORT=29741 RANK=0 WORLD_SIZE=1 python scripts/gather_overhead.py
"""
import importlib
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
m = importlib.import_module("cs201_sah-bvh_ray_tracer_amd")
shard = importlib.import_module("cs201_sah-bvh_ray_tracer_amd.shard")


def main():
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    W, H, batch, launches = 1920, 1080, 4, 5
    s = m.create_random_spheres(10000, 1)
    b = m.build_bvh(s)
    rs = [m.Renderer(0) for _ in range(8)]
    for r in rs:
        r.upload(s, b)
        r.set_option(m.abi.OPT_BOUNCE_BLOCKS, 384)
    sf = shard.ShardedFrame(rs[0], W, H, samples=batch, renderers=rs, accum=False)
    cam = m.default_camera()
    out = {}
    for gather in (False, True):
        def launch(f0):
            sf.render_local(cam, sf.desc(seed=1, sample=f0, samples=batch))
            if gather:
                sf.gather(every=1)
        for f in range(0, 2 * launches * batch, batch):
            launch(f)
        torch.cuda.synchronize()
        host, gpu = [], []
        for rep in range(5):
            t0 = time.perf_counter()
            for k in range(launches):
                launch(k * batch)
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            host.append((t1 - t0) / launches * 1e3)
            gpu.append((t2 - t0) / launches * 1e3)
        key = "with_gather" if gather else "render_only"
        out[key] = {"host_enqueue_ms_per_launch": round(sorted(host)[2], 4),
                    "wall_ms_per_launch": round(sorted(gpu)[2], 4)}
    out["note"] = ("world-1 nccl group: the gather moves this rank's own 4-frame slab (a whole frame's rows here, "
                   "1/8 of them at N = 8); the host cost per call is what matters")
    print(json.dumps(out), flush=True)
    dist.destroy_process_group()
    for r in rs:
        r.close()


if __name__ == "__main__":
    main()
