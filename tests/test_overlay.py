"""The BVH debug overlay (bvh_visualiser.c:16-126, main.c's 'o' view) as a
GPU line raster (mirt_bvh_overlay). The reference draws through SDL (its
rasterisation is the backend's; the file is marked "NOT WORKING"), so there
is no reference framebuffer to pin: CPU tests check the oracle's restatement
for properties -- every lit pixel lies on a projected box edge (within the
one-pixel offsets of draw_debug_line), a pixel's colour is the depth colour
of a node drawn over it, the first level alone is the root box in the root's
colour -- and the GPU test checks the HIP raster against that restatement
byte for byte."""
import numpy as np
import pytest


def _setup(mirt, oracle, n, cam_i=0, small=None):
    s = oracle.render_scene(1, n)
    t = oracle.build(s)
    cam = mirt.default_camera()
    if cam_i == 1:
        cam = mirt.abi.Camera.from_numpy(small["cameras"][1])
    return s, t, cam


def _project(cam, p, W, H):
    """world_to_screen in float32 (bvh_visualiser.c:16-41)."""
    f32 = np.float32
    pos = np.array([cam.position.x, cam.position.y, cam.position.z], f32)
    fw = np.array([cam.forward.x, cam.forward.y, cam.forward.z], f32)
    rt = np.array([cam.right.x, cam.right.y, cam.right.z], f32)
    up = np.array([cam.up.x, cam.up.y, cam.up.z], f32)
    t = np.asarray(p, f32) - pos
    z = f32(f32(t[0] * fw[0]) + f32(t[1] * fw[1])) + f32(t[2] * fw[2])
    if not z > f32(0.1):
        return None
    x = f32(f32(t[0] * rt[0]) + f32(t[1] * rt[1])) + f32(t[2] * rt[2])
    y = f32(f32(t[0] * up[0]) + f32(t[1] * up[1])) + f32(t[2] * up[2])
    fov = f32(np.float64(cam.fov) * (np.pi / 180.0))
    hh = f32(np.tan(f32(fov / f32(2))))
    hw = f32(f32(W) / f32(H)) * hh
    sx = (x / (z * hw * f32(2)) + f32(0.5)) * f32(W)
    sy = (-y / (z * hh * f32(2)) + f32(0.5)) * f32(H)
    if sx < -W or sx > 2 * W or sy < -H or sy > 2 * H:
        return None
    return int(sx), int(sy)


def _depth_colour(d):
    return (255 - (d * 40) % 200, (d * 80) % 200, (d * 120) % 200, 180)


def test_overlay_root_level_is_the_root_box(mirt, oracle):
    """max_levels = 1: only the root box, in the root's colour (255, 0, 0,
    180); its projected visible corners are lit."""
    W, H = 160, 90
    s, t, cam = _setup(mirt, oracle, 100)
    img = oracle.bvh_overlay(t, cam, W, H, 1)
    lit = (img != np.array([0, 0, 0, 255], np.uint8)).any(-1)
    assert lit.sum() > 50
    assert (img[lit] == np.array(_depth_colour(0), np.uint8)).all()
    root = oracle.flatten(t)[0]
    lo, hi = root["bmin"], root["bmax"]
    for k in range(8):
        c = [hi[0] if k in (1, 2, 5, 6) else lo[0], hi[1] if k in (2, 3, 6, 7) else lo[1], hi[2] if k >= 4 else lo[2]]
        p = _project(cam, c, W, H)
        if p and 0 <= p[0] < W and 0 <= p[1] < H:
            assert lit[p[1], p[0]], (k, p)
    oracle.free(t)


@pytest.mark.parametrize("levels", [3, -1])
def test_overlay_pixels_lie_on_projected_edges(mirt, oracle, levels):
    """Every lit pixel is within one pixel (the offset lines) of the
    segment between the projected endpoints of some drawn edge, and its
    colour is the depth colour of such an edge's node."""
    W, H = 160, 90
    s, t, cam = _setup(mirt, oracle, 60)
    img = oracle.bvh_overlay(t, cam, W, H, levels)
    flat = oracle.flatten(t)
    depth = np.zeros(len(flat), np.int32)
    skip = flat["skip"] & mirt.abi.SKIP_MASK
    for i in range(len(flat)):
        if flat["sphere"][i] < 0:
            depth[i + 1] = depth[skip[i + 1]] = depth[i] + 1
    edges = [(0, 1), (1, 2), (2, 3), (3, 0), (4, 5), (5, 6), (6, 7), (7, 4), (0, 4), (1, 5), (2, 6), (3, 7)]
    segs = []   # (x0, y0, x1, y1, colour)
    for i, nd in enumerate(flat):
        if levels >= 0 and depth[i] >= levels:
            continue
        lo, hi = nd["bmin"], nd["bmax"]
        corners = [[hi[0] if k in (1, 2, 5, 6) else lo[0], hi[1] if k in (2, 3, 6, 7) else lo[1],
                    hi[2] if k >= 4 else lo[2]] for k in range(8)]
        pts = [_project(cam, c, W, H) for c in corners]
        for a, b in edges:
            if pts[a] and pts[b]:
                segs.append((*pts[a], *pts[b], _depth_colour(int(depth[i]))))
    assert segs
    ys, xs = np.nonzero((img != np.array([0, 0, 0, 255], np.uint8)).any(-1))
    assert len(xs) > 100
    S = np.array([g[:4] for g in segs], np.float64)
    cols = np.array([g[4] for g in segs], np.uint8)
    for x, y in zip(xs, ys):
        ax, ay, bx, by = S[:, 0], S[:, 1], S[:, 2], S[:, 3]
        dx, dy = bx - ax, by - ay
        L2 = np.maximum(dx * dx + dy * dy, 1e-12)
        u = np.clip(((x - ax) * dx + (y - ay) * dy) / L2, 0, 1)
        dist = np.hypot(ax + u * dx - x, ay + u * dy - y)
        near = dist <= 1.0 + 0.75      # one-pixel offset + Bresenham's half-pixel rounding
        assert near.any(), (x, y)
        assert (cols[near] == img[y, x]).all(axis=1).any(), (x, y, img[y, x])
    oracle.free(t)


@pytest.mark.gpu
@pytest.mark.parametrize("W,H,n,levels,cam_i", [(160, 90, 100, -1, 0), (320, 180, 1000, 4, 0),
                                                 (320, 180, 1000, -1, 1), (640, 360, 10000, 6, 0)])
def test_gpu_overlay_matches_oracle(gpu, mirt, oracle, small, W, H, n, levels, cam_i):
    s, t, cam = _setup(mirt, oracle, n, cam_i, small)
    ref = oracle.bvh_overlay(t, cam, W, H, levels)
    oracle.free(t)
    s2 = mirt.create_random_spheres(n, 1)
    b = mirt.build_bvh(s2)
    gpu.upload(s2, b)
    got = gpu.bvh_overlay(cam, W, H, levels)
    assert (got == ref).all(), int((got != ref).any(-1).sum())
