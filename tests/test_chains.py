"""MIRT_OPT_CHAINS (the chain handoff between bounce launches, render.hip
ContRec / defer_chain): once a bounce wave finds the queue dry, a chain that
goes on to its next level is appended to a continuation queue that the
frame's next bounce launch takes -- the same per-pixel arithmetic
(renderer.c:21-77 per level, the pixel's RNG draws in order, the colour
stack folded innermost-first), executed by other lanes. Checked against the
golden frames of the unmodified reference (tests/golden/golden.json,
full.json) and the oracle (every depth the colour stack holds, accumulation,
shards, frames in flight)."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, sha
from test_gpu_parity import _scene

pytestmark = pytest.mark.gpu


def _chains(gpu, mirt, on):
    gpu.set_option(mirt.abi.OPT_CHAINS, 1 if on else 0)


def test_chains_option_roundtrip(gpu, mirt):
    try:
        _chains(gpu, mirt, True)
        assert gpu.get_option(mirt.abi.OPT_CHAINS) == 1
        with pytest.raises(mirt.MirtError):
            gpu.set_option(mirt.abi.OPT_CHAINS, 2)
    finally:
        _chains(gpu, mirt, False)
    assert gpu.get_option(mirt.abi.OPT_CHAINS) == 0


@pytest.mark.parametrize("threshold,blocks,drain", [(20, 0, 1), (20, 384, 1), (40, 64, 1), (20, 0, 0)])
def test_chains_golden_1080p(gpu, mirt, golden, threshold, blocks, drain):
    """The metric's frame (1080p, 10k spheres, depth 5) with the handoff, at
    the full grid, the bench's 384 workgroups, a small grid (most chains
    handed over) and without the quad drain."""
    abi = mirt.abi
    s, b = _scene(mirt, "render", 10000)
    gpu.upload(s, b)
    cam = mirt.default_camera()
    try:
        _chains(gpu, mirt, True)
        gpu.set_option(abi.OPT_BOUNCE_THRESHOLD, threshold)
        gpu.set_option(abi.OPT_BOUNCE_BLOCKS, blocks)
        gpu.set_option(abi.OPT_QUAD_DRAIN, drain)
        img = gpu.render_frame(cam, 1920, 1080, depth=5, seed=1)
    finally:
        _chains(gpu, mirt, False)
        gpu.set_option(abi.OPT_BOUNCE_THRESHOLD, 20)
        gpu.set_option(abi.OPT_BOUNCE_BLOCKS, 0)
        gpu.set_option(abi.OPT_QUAD_DRAIN, 1)
    assert sha(img) == golden["frames"]["1920x1080_render10000_d5_m1_b1_s1_c0_step1"]["sha"]


def _full_cases():
    path = os.path.join(GOLDEN, "full.json")
    if not os.path.exists(path):
        return {}
    with open(path) as f:
        return {k: v for k, v in json.load(f)["cases"].items() if v["depth"] >= 3}


FULL = _full_cases()


@pytest.mark.parametrize("key", sorted(FULL))
def test_chains_full_frames(gpu, mirt, key):
    """BASELINE configs[2]-[4] with the handoff (4K/1M: four jittered samples
    in one launch) against the reference's whole-frame SHAs."""
    import torch
    c = FULL[key]
    s = mirt.create_random_spheres(c["n"], c["seed"]) if c["kind"] == "render" else \
        mirt.create_benchmark_spheres(c["n"], c["seed"])
    gpu.upload(s, mirt.build_bvh(s))
    W, H, S = c["W"], c["H"], c["samples"]
    fd = mirt.frame_desc(W, H, depth=c["depth"], seed=c["seed"], samples=S, jitter=c["jitter"])
    out = torch.zeros((S, H, W), dtype=torch.int32, device="cuda")
    try:
        _chains(gpu, mirt, True)
        gpu.render_frame_device(mirt.default_camera(), fd, out.data_ptr(), None,
                                torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
    finally:
        _chains(gpu, mirt, False)
    img = out.cpu().numpy().view(np.uint8).reshape(S, H, W, 4)
    for k in range(S):
        assert hashlib.sha256(img[k].tobytes()).hexdigest() == c["frame_sha"][k], (key, k)


@pytest.mark.parametrize("depth", [3, 4, 6, 8])
def test_chains_depths_vs_oracle(gpu, mirt, oracle, small, depth):
    """Every colour-stack depth a continuation carries (depth 8: six rows),
    fresh and accumulating, whole frame and shard 1 of 3, at a grid small
    enough that most chains are handed over, against the oracle."""
    abi = mirt.abi
    s, b = _scene(mirt, "render", 1000)
    gpu.upload(s, b)
    cam = mirt.default_camera()
    W, H = 160, 90
    t = oracle.build(small["render_1000_1_pre"].copy())
    try:
        _chains(gpu, mirt, True)
        gpu.set_option(abi.OPT_BOUNCE_BLOCKS, 8)
        for shard, world in ((0, 1), (1, 3)):
            acc = np.zeros(W * H * 3, np.float32)
            rows = mirt.shard_rows(mirt.frame_desc(W, H, shard=shard, num_shards=world))
            for k in range(3):
                got = gpu.render_frame(cam, W, H, depth=depth, seed=4, sample=k, accumulate=k > 0, frames=k + 1,
                                       shard=shard, num_shards=world)
                col = oracle.render(cam, W, H, s, t, depth=depth, mode=1, seed=4, sample=k)
                ref = oracle.accumulate(col, acc, k == 0, k + 1).reshape(H, W, 4)
                assert (got == ref[rows]).all(), (depth, shard, k)
            # three frames in flight in one launch == the accumulating loop
            one = gpu.render_frame(cam, W, H, depth=depth, seed=4, sample=0, samples=3, shard=shard,
                                   num_shards=world)
            assert (one == got).all(), (depth, shard)
    finally:
        _chains(gpu, mirt, False)
        gpu.set_option(abi.OPT_BOUNCE_BLOCKS, 0)
        oracle.free(t)


def test_chains_off_below_depth3(gpu, mirt, golden):
    """Depth 1 and 2 have nothing to hand over (depth 2: one bounce level):
    the option leaves them on the one-launch path, frames unchanged."""
    s, b = _scene(mirt, "render", 10000)
    gpu.upload(s, b)
    cam = mirt.default_camera()
    ref = {d: gpu.render_frame(cam, 640, 360, depth=d, seed=1) for d in (1, 2)}
    try:
        _chains(gpu, mirt, True)
        for d in (1, 2):
            assert (gpu.render_frame(cam, 640, 360, depth=d, seed=1) == ref[d]).all(), d
    finally:
        _chains(gpu, mirt, False)
