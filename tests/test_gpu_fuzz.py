"""Seeded random cameras and scenes: the HIP frame against the oracle's
(renderer.c:21-77 per pixel of main.c:356-366, with get_camera_ray ray.c:17-32
and camera_update), byte for byte.

The golden frames pin the default camera and camera 1; these cases move the
camera inside and around the sphere cloud, along the axes (rays with zero
direction components, which hit.c:54-57 treats specially), through ragged
tile edges (W, H not multiples of the 8x8 tile) and over both scene
generators, so that the camera packets, the deferred zero-component rays, the
bounce queue and the four-wide walk are all exercised off the tested views.
"""
import os

import numpy as np
import pytest

# MIRT_FUZZ_CASES raises the count for a longer soak (profiles/r03zh: 512 per
# scene kind); the default keeps the suite to seconds
CASES = int(os.environ.get("MIRT_FUZZ_CASES", "16"))


def _cameras(mirt, rng):
    cams = []
    for i in range(CASES):
        cam = mirt.default_camera()
        if i == 0:
            cam.position = mirt.abi.Vec3(0.0, 0.0, 0.0)          # inside the cloud, default axes
        elif i == 1:
            cam.position = mirt.abi.Vec3(0.0, 4.0, -60.0)
            cam.yaw = np.float32(0.0)                            # looking down +z
            mirt.camera_update(cam)
        elif i == 2:
            cam.yaw = np.float32(-np.pi / 2)                     # along an axis from the side
            cam.position = mirt.abi.Vec3(60.0, 0.0, 0.0)
            mirt.camera_update(cam)
        else:
            p = rng.uniform(-70.0, 70.0, 3)
            cam.position = mirt.abi.Vec3(*map(float, p))
            cam.yaw = np.float32(rng.uniform(-np.pi, np.pi))
            cam.pitch = np.float32(rng.uniform(-1.4, 1.4))
            cam.fov = float(rng.uniform(20.0, 90.0))
            mirt.camera_update(cam)
        cams.append(cam)
    return cams


@pytest.fixture(scope="module")
def scenes(mirt):
    return {"render": mirt.create_random_spheres(3000, 11),
            "bench": mirt.create_benchmark_spheres(4000, 5, world_size=120.0)}


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["render", "bench"])
def test_random_cameras_match_oracle(gpu, mirt, oracle, scenes, kind):
    rng = np.random.default_rng(2024 if kind == "render" else 7)
    s = scenes[kind].copy()
    s2 = s.copy()
    gpu.upload(s, mirt.build_bvh(s))
    t = oracle.build(s2)
    try:
        sizes = [(96, 54), (77, 45), (130, 9)]
        for i, cam in enumerate(_cameras(mirt, rng)):
            W, H = sizes[i % len(sizes)]
            depth = 5 if i % 3 else 3
            img = gpu.render_frame(cam, W, H, depth=depth, seed=1 + i)
            ref = oracle.render(cam, W, H, s2, t, depth=depth, use_bvh=True, mode=1, seed=1 + i)
            bad = int((img != ref).any(-1).sum())
            assert bad == 0, f"{kind} camera {i} ({W}x{H}, depth {depth}): {bad} pixels differ"
    finally:
        oracle.free(t)
