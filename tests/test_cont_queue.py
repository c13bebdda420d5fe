"""The bounce pass's continuation queue (MIRT_OPT_CONT_QUEUE, render.hip
bounce_kernel<..., CQ>): chains that start a new level after the queue ran
dry are handed to waiting waves and walked with the whole wave. It moves
work, never results: every frame must equal the queue-off frame and the
reference's goldens. The blocking call uses it (a frame alone on
the chip) with option 1 (default 0: measured slower); option 2
forces it for frames in flight too."""
import hashlib

import numpy as np
import pytest

GOLD = "1920x1080_render10000_d5_m1_b1_s1_c0_step1"


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.fixture(scope="module")
def scene10k(mirt):
    s = mirt.create_random_spheres(10000, 1)
    return s, mirt.build_bvh(s)


@pytest.mark.gpu
def test_cont_queue_default_off(gpu, mirt):
    """Measured slower than the drain it would replace: off
    unless asked for."""
    assert gpu.get_option(mirt.abi.OPT_CONT_QUEUE) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [1, 2])
def test_cont_queue_golden_1080p(gpu, mirt, golden, scene10k, mode):
    s, b = scene10k
    gpu.upload(s, b)
    try:
        gpu.set_option(mirt.abi.OPT_CONT_QUEUE, mode)
        for _ in range(3):
            assert sha(gpu.render_frame(mirt.default_camera(), 1920, 1080, depth=5, seed=1)) == \
                golden["frames"][GOLD]["sha"]
    finally:
        gpu.set_option(mirt.abi.OPT_CONT_QUEUE, 0)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,n,depth,W,H", [("render", 100000, 5, 640, 360), ("render", 1000, 8, 160, 90),
                                               ("bench", 20000, 5, 320, 180), ("render", 10000, 3, 77, 45),
                                               ("render", 10000, 2, 333, 187)])
def test_cont_queue_equals_queue_off(gpu, mirt, kind, n, depth, W, H):
    s = mirt.create_random_spheres(n, 1) if kind == "render" else mirt.create_benchmark_spheres(n, 1)
    b = mirt.build_bvh(s)
    gpu.upload(s, b)
    cam = mirt.default_camera()
    if kind == "bench":
        cam.position.z = 900.0
    try:
        gpu.set_option(mirt.abi.OPT_CONT_QUEUE, 0)
        want = [gpu.render_frame(cam, W, H, depth=depth, seed=s_, sample=k) for s_, k in ((1, 0), (5, 3))]
        for mode in (1, 2):
            gpu.set_option(mirt.abi.OPT_CONT_QUEUE, mode)
            got = [gpu.render_frame(cam, W, H, depth=depth, seed=s_, sample=k) for s_, k in ((1, 0), (5, 3))]
            for g, w in zip(got, want):
                assert (g == w).all(), mode
    finally:
        gpu.set_option(mirt.abi.OPT_CONT_QUEUE, 0)


@pytest.mark.gpu
def test_cont_queue_frames_in_flight(gpu, mirt, scene10k):
    """Option 2 on four lanes of frames in flight (each launch's waiting waves
    hold their slots until its last chain ends): still the one-context frames."""
    s, b = scene10k
    W, H, F = 640, 360, 8
    cam = mirt.default_camera()
    bufs = [mirt.HostBuffer((H, W, 4)) for _ in range(F)]
    try:
        with mirt.MultiRenderer([0], lanes=4) as m:
            m.upload(s, b)
            m.set_option(mirt.abi.OPT_CONT_QUEUE, 2)
            for k in range(F):
                m.render_frames_async(cam, mirt.frame_desc(W, H, depth=5, seed=2, sample=k), [bufs[k]])
            m.wait()
            got = [x.array.copy() for x in bufs]
    finally:
        for x in bufs:
            x.close()
    gpu.upload(s, b)
    gpu.set_option(mirt.abi.OPT_CONT_QUEUE, 0)
    try:
        for k in range(F):
            assert (got[k] == gpu.render_frame(cam, W, H, depth=5, seed=2, sample=k)).all(), k
    finally:
        gpu.set_option(mirt.abi.OPT_CONT_QUEUE, 0)
