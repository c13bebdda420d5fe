"""mirt_multi over DISTINCT devices (the n-GPU RCCL exchange): the
golden 1080p / 10k depth-5 frame through the RCCL gather (ncclSend from
devices 1..n-1, ncclRecv on device 0) and through host-direct delivery, with
one lane and with lanes in flight carrying several frames per launch. Runs on
a node with 2 or more GPUs (up to 8 of them); on the one-GPU test box every
case skips -- the same geometry is covered there by same-device ranks
(tests/test_multi.py)."""
import hashlib

import numpy as np
import pytest

GOLD = "1920x1080_render10000_d5_m1_b1_s1_c0_step1"


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def n_devices():
    import torch
    return torch.cuda.device_count()   # counts devices without initialising the runtime


@pytest.fixture(scope="module")
def devices():
    n = n_devices()
    if n < 2:
        pytest.skip(f"{n} GPU(s) visible: the distinct-device exchange needs 2 or more")
    return list(range(min(n, 8)))


@pytest.fixture(scope="module")
def scene10k(mirt):
    s = mirt.create_random_spheres(10000, 1)
    return s, mirt.build_bvh(s)


@pytest.mark.gpu
@pytest.mark.parametrize("direct", [False, True])
def test_distinct_devices_golden_one_lane(mirt, golden, scene10k, devices, direct):
    s, b = scene10k
    with mirt.MultiRenderer(devices, host_direct=direct) as m:
        assert m.size == len(devices)
        assert m.backend == "rccl" and m.delivery == ("host-direct" if direct else "gather")
        m.upload(s, b)
        for _ in range(2):
            img = m.render_frame(mirt.default_camera(), 1920, 1080, depth=5, seed=1)
            assert sha(img) == golden["frames"][GOLD]["sha"]


@pytest.mark.gpu
@pytest.mark.parametrize("direct", [False, True])
def test_distinct_devices_lanes_in_flight(gpu, mirt, scene10k, devices, direct):
    """Three lanes, launches of four successive fresh frames (bench.py's
    N >= 4 schedule): every frame equals one context's frame of its sample."""
    s, b = scene10k
    W, H, F, batch = 640, 360, 12, 4
    cam = mirt.default_camera()
    bufs = [mirt.HostBuffer((H, W, 4)) for _ in range(F)]
    try:
        with mirt.MultiRenderer(devices, lanes=3, host_direct=direct) as m:
            m.upload(s, b)
            for f0 in range(0, F, batch):
                m.render_frames_async(cam, mirt.frame_desc(W, H, depth=5, seed=3, sample=f0), bufs[f0:f0 + batch])
            m.wait()
            got = [x.array.copy() for x in bufs]
    finally:
        for x in bufs:
            x.close()
    gpu.upload(s, b)
    for j in range(F):
        assert (got[j] == gpu.render_frame(cam, W, H, depth=5, seed=3, sample=j)).all(), j
