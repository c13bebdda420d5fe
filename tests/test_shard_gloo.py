"""The N>1 path on CPU: world_size 2 and 3 over gloo. Each rank produces its
row-block slab (here with the oracle standing in for the GPU kernel -- this
test covers the shard geometry, the gather and the de-interleave, which are
the same code bench.py runs over RCCL), rank 0 gathers and assembles, and the
frame must equal the single-process frame byte for byte."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W, H, RB = 96, 61, 8


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, result_path, frames=1):
    sys.path.insert(0, ROOT)
    import importlib

    import torch.distributed as dist

    mirt = importlib.import_module("cs201_sah-bvh_ray_tracer_amd")
    shard = importlib.import_module("cs201_sah-bvh_ray_tracer_amd.shard")
    from oracle.lib import Oracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    o = Oracle()
    s = o.render_scene(1, 500)
    t = o.build(s)
    cam = mirt.default_camera()
    fd = mirt.frame_desc(W, H, depth=5, seed=2, row_block=RB, shard=rank, num_shards=world)
    rows = mirt.shard_rows(fd)
    slab = np.zeros((frames, shard.slab_rows(H, RB, world), W, 4), np.uint8)
    for j in range(frames):
        slab[j, :len(rows)] = o.render(cam, W, H, s, t, depth=5, mode=1, seed=2, sample=j, rows=rows, threads=1)
    st = torch.from_numpy(slab.view(np.int32).reshape(frames, -1, W))
    # one frame: a (rows, W) slab; several (bench.py's multi-frame launches): (frames, rows, W)
    frame = shard.gather_frame(st[0] if frames == 1 else st, H, RB)
    if rank == 0:
        ok = shape = 1
        for j in range(frames):
            full = o.render(cam, W, H, s, t, depth=5, mode=1, seed=2, sample=j, threads=1)
            got = shard.as_rgba(frame if frames == 1 else frame[j]).numpy()
            ok &= int((got == full).all())
            shape &= int(got.shape == full.shape)
        np.save(result_path, np.array([ok, shape]))
    o.free(t)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,frames", [(2, 1), (3, 1), (2, 3)])
def test_gloo_gather_matches_single_frame(tmp_path, world, frames):
    res = str(tmp_path / "res.npy")
    mp.spawn(_worker, args=(world, _free_port(), res, frames), nprocs=world, join=True)
    ok = np.load(res)
    assert ok.tolist() == [1, 1]
