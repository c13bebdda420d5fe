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


@pytest.mark.parametrize("key", sorted(CASES))
def test_gpu_full_frames(gpu, mirt, key):
    import torch
    c = CASES[key]
    s = mirt.create_random_spheres(c["n"], c["seed"]) if c["kind"] == "render" else \
        mirt.create_benchmark_spheres(c["n"], c["seed"])
    b = mirt.build_bvh(s)                 # [0, n), depth 0
    gpu.upload(s, b)
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
