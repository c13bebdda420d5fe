"""BASELINE configs[2]-[4] on WHOLE frames against the reference itself:
tests/golden/full.json holds the SHA-256 of every full RGBA8 frame the
unmodified reference renders (oracle/_ref, renderer.c:21-77 under
main.c:358-374's pixel loop; make_golden_full.py) --

  configs[2]  1920x1080, 100,000 random spheres, depth 5 and depth 1
  configs[3]  3840x2160, 10,000 random spheres, depth 5
  configs[4]  3840x2160, 1,000,000 benchmark spheres, 4 jittered samples

-- and a 16-hex SHA-256 prefix per 8-row block, so a mismatch names its
rows. GPU: every sample of a case in ONE launch (frames in flight, raw
slabs), each compared whole."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _cases():
    path = os.path.join(GOLDEN, "full.json")
    if not os.path.exists(path):
        return {}
    with open(path) as f:
        return json.load(f)["cases"]


CASES = _cases()


def test_full_frame_goldens_cover_baseline_configs():
    assert {(c["W"], c["H"], c["n"], c["depth"], c["samples"]) for c in CASES.values()} >= {
        (1920, 1080, 100000, 5, 1), (1920, 1080, 100000, 1, 1), (3840, 2160, 10000, 5, 1),
        (3840, 2160, 1000000, 5, 4)}


@pytest.mark.parametrize("order,walk", [(0, 0), (1, 0), (0, 1)])
@pytest.mark.parametrize("key", sorted(CASES))
def test_gpu_full_frames(gpu, mirt, key, order, walk):
    """`order`: MIRT_OPT_NODE_ORDER of the uploaded four-wide tree
    (breadth-first numbering, or depth-first sibling groups); `walk`:
    MIRT_OPT_PRIMARY_WALK (camera rays as packets, or per lane four-wide):
    the frames must not depend on either."""
    import torch
    c = CASES[key]
    s = mirt.create_random_spheres(c["n"], c["seed"]) if c["kind"] == "render" else \
        mirt.create_benchmark_spheres(c["n"], c["seed"])
    b = mirt.build_bvh(s)                 # [0, n), depth 0
    gpu.set_option(mirt.abi.OPT_NODE_ORDER, order)
    try:
        gpu.upload(s, b)
    finally:
        gpu.set_option(mirt.abi.OPT_NODE_ORDER, 0)
    gpu.set_option(mirt.abi.OPT_PRIMARY_WALK, walk)
    try:
        _render_and_check(gpu, mirt, key, c)
    finally:
        gpu.set_option(mirt.abi.OPT_PRIMARY_WALK, 0)


def _render_and_check(gpu, mirt, key, c):
    import torch
    W, H, S = c["W"], c["H"], c["samples"]
    fd = mirt.frame_desc(W, H, depth=c["depth"], seed=c["seed"], samples=S, jitter=c["jitter"])
    out = torch.zeros((S, H, W), dtype=torch.int32, device="cuda")
    gpu.render_frame_device(mirt.default_camera(), fd, out.data_ptr(), None, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    img = out.cpu().numpy().view(np.uint8).reshape(S, H, W, 4)
    B = 8
    for k in range(S):
        got = hashlib.sha256(img[k].tobytes()).hexdigest()
        if got != c["frame_sha"][k]:
            bad = [y for i, y in enumerate(range(0, H, B))
                   if hashlib.sha256(img[k][y:y + B].tobytes()).hexdigest()[:16] != c["block_sha16"][k][i]]
            pytest.fail(f"{key} sample {k}: {len(bad)} of {len(c['block_sha16'][k])} 8-row blocks differ, "
                        f"first rows {bad[:8]}")


@pytest.mark.parametrize("walk", [0, 1])
def test_gpu_primary_walk_golden_1080p_10k(gpu, mirt, golden, walk):
    """The metric's frame with the camera rays walked as packets or per lane
    (MIRT_OPT_PRIMARY_WALK), depth 5 and depth 1 (the camera kernel alone)."""
    s = mirt.create_random_spheres(10000, 1)
    gpu.upload(s, mirt.build_bvh(s))
    gpu.set_option(mirt.abi.OPT_PRIMARY_WALK, walk)
    try:
        assert gpu.get_option(mirt.abi.OPT_PRIMARY_WALK) == walk
        for d, mode in ((5, 1), (1, 0)):    # (mode: the oracle's RNG contract; depth 1 draws nothing)
            img = gpu.render_frame(mirt.default_camera(), 1920, 1080, depth=d, seed=1)
            assert hashlib.sha256(img.tobytes()).hexdigest() == \
                golden["frames"][f"1920x1080_render10000_d{d}_m{mode}_b1_s1_c0_step1"]["sha"], d
    finally:
        gpu.set_option(mirt.abi.OPT_PRIMARY_WALK, 0)


@pytest.mark.parametrize("order", [0, 1])
def test_gpu_node_order_golden_1080p_10k(gpu, mirt, golden, order):
    """The metric's frame (1080p / 10k, depth 5, tests/golden/golden.json)
    with either four-wide tree layout, and both layouts agree on the
    per-ray batch (mirt_intersect_rays through the quad walk)."""
    s = mirt.create_random_spheres(10000, 1)
    b = mirt.build_bvh(s)
    gpu.set_option(mirt.abi.OPT_NODE_ORDER, order)
    try:
        gpu.upload(s, b)
    finally:
        gpu.set_option(mirt.abi.OPT_NODE_ORDER, 0)
    assert gpu.get_option(mirt.abi.OPT_NODE_ORDER) == 0
    img = gpu.render_frame(mirt.default_camera(), 1920, 1080, depth=5, seed=1)
    assert hashlib.sha256(img.tobytes()).hexdigest() == golden["frames"]["1920x1080_render10000_d5_m1_b1_s1_c0_step1"]["sha"]
    rng = np.random.default_rng(5)
    rays = np.zeros(4096, mirt.abi.RAY)
    rays["origin"] = rng.uniform(-60, 60, (4096, 3)).astype(np.float32)
    rays["direction"] = rng.normal(size=(4096, 3)).astype(np.float32)
    hits = gpu.closest_hit(rays)
    gpu.upload(s, b)                      # the default layout
    ref = gpu.closest_hit(rays)
    assert (hits == ref).all()
