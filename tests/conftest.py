import hashlib
import importlib
import json
import os
import sys

import numpy as np
import pytest
# torch before libmirt.so: both need libamdhip64.so.7, and the process must
# hold ONE HIP runtime (torch's) for device pointers and streams from torch
# to be valid in libmirt -- as in bench.py, which imports torch first
import torch  # noqa: F401

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libmirt.so on cuda:0)")


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.fixture(scope="session")
def mirt():
    return importlib.import_module("cs201_sah-bvh_ray_tracer_amd")


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(GOLDEN, "golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def small():
    with np.load(os.path.join(GOLDEN, "small.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def oracle():
    from oracle.lib import Oracle
    return Oracle()


@pytest.fixture(scope="session")
def gpu(mirt):
    """One device context on cuda:0 for the whole session (no CPU fallback:
    raises if libmirt.so or the GPU is missing)."""
    r = mirt.Renderer(0)
    yield r
    r.close()


def parse_frame_key(key):
    """'160x90_render100_d5_m1_b1_s1_c0_step1' -> dict"""
    res, scene, d, m, b, s, c, step = key.split("_")
    W, H = map(int, res.split("x"))
    kind = "render" if scene.startswith("render") else "bench"
    n = int(scene[len(kind):])
    return dict(W=W, H=H, kind=kind, n=n, depth=int(d[1:]), mode=int(m[1:]), use_bvh=bool(int(b[1:])),
                seed=int(s[1:]), cam=int(c[1:]), step=int(step[4:]))
