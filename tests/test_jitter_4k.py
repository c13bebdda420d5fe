"""BASELINE configs[3] / configs[4]: 4K frames, the 1M-sphere benchmark
scene and jittered accumulation samples, against tests/golden/jitter.json
(made by make_golden_jitter.py from the unmodified reference through
oracle/_ref). CPU: the oracle restatement; GPU: the HIP path, per sample
(one launch of `samples` frames, raw slabs) and accumulated."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, sha


@pytest.fixture(scope="module")
def jgold():
    with open(os.path.join(GOLDEN, "jitter.json")) as f:
        return json.load(f)


def _scene(mirt, kind, n, seed):
    s = mirt.create_random_spheres(n, seed) if kind == "render" else mirt.create_benchmark_spheres(n, seed)
    b = mirt.build_bvh(s)     # [0, n), depth 0
    return s, b


def test_oracle_jitter_frames(mirt, oracle, jgold):
    """The oracle's jittered / 4K samples equal the reference's (cases up to
    20k spheres; the 1M-sphere case runs on the GPU side)."""
    cam = mirt.default_camera()
    for key, c in jgold["cases"].items():
        if c["n"] > 20000:
            continue
        s = oracle.render_scene(c["seed"], c["n"]) if c["kind"] == "render" else oracle.bench_scene(c["seed"], c["n"])
        t = oracle.build(s)
        rows = None if c["rows"] is None else np.array(c["rows"], np.int32)
        for k, want in enumerate(c["sample_sha"]):
            img = oracle.render(cam, c["W"], c["H"], s, t, depth=c["depth"], mode=1, seed=c["seed"], sample=k,
                                rows=rows, jitter=c["jitter"])
            assert sha(img) == want, (key, k)
        oracle.free(t)


@pytest.mark.gpu
def test_gpu_jitter_frames(gpu, mirt, jgold):
    """Every case: all samples in ONE launch (frames in flight, raw slabs)
    equal the reference's per-sample rows."""
    import torch
    cam = mirt.default_camera()
    for key, c in jgold["cases"].items():
        s, b = _scene(mirt, c["kind"], c["n"], c["seed"])
        gpu.upload(s, b)
        W, H, S = c["W"], c["H"], len(c["sample_sha"])
        fd = mirt.frame_desc(W, H, depth=c["depth"], seed=c["seed"], samples=S, jitter=c["jitter"])
        out = torch.zeros((S, H, W), dtype=torch.int32, device="cuda")
        stream = torch.cuda.current_stream()
        gpu.render_frame_device(cam, fd, out.data_ptr(), None, stream.cuda_stream)
        torch.cuda.synchronize()
        img = out.cpu().numpy().view(np.uint8).reshape(S, H, W, 4)
        rows = slice(None) if c["rows"] is None else np.array(c["rows"])
        for k, want in enumerate(c["sample_sha"]):
            assert sha(img[k][rows]) == want, (key, k)


@pytest.mark.gpu
def test_gpu_jitter_accumulation(gpu, mirt, oracle, jgold):
    """4 jittered samples accumulated in one call == the oracle's
    accumulation of its per-sample frames (main.c:379-408)."""
    c = jgold["cases"]["320x180_bench1000_s1_d5_j1"]
    s, b = _scene(mirt, "bench", c["n"], c["seed"])
    gpu.upload(s, b)
    cam = mirt.default_camera()
    W, H = c["W"], c["H"]
    got = gpu.render_frame(cam, W, H, depth=5, seed=c["seed"], samples=4, jitter=True)
    s2 = oracle.bench_scene(c["seed"], c["n"])
    t = oracle.build(s2)
    acc = np.zeros(W * H * 3, np.float32)
    for k in range(4):
        col = oracle.render(cam, W, H, s2, t, depth=5, mode=1, seed=c["seed"], sample=k, jitter=True)
        ref = oracle.accumulate(col, acc, k == 0, k + 1).reshape(H, W, 4)
    oracle.free(t)
    assert (got == ref).all()
