"""Pin the oracle (oracle/oracle.c, the CPU restatement) to the reference.

Every vector in tests/golden/ was produced by the UNMODIFIED reference
sources (tests/golden/make_golden.py); this file checks the restatement
against all of them, bit for bit. CPU only.
"""
import ctypes as C

import numpy as np
import pytest

from conftest import parse_frame_key, sha
from oracle.lib import abi


def test_glibc_rand_streams(oracle, golden):
    for seed, vals in golden["rand"].items():
        oracle.L.o_srand(int(seed))
        assert [oracle.L.o_libc_rand() for _ in range(len(vals))] == vals


def test_contract_draws(oracle, golden):
    for seed, px, smp, k, v in golden["contract"]:
        assert oracle.contract_draw(seed, px, smp, k) == v
        assert 0 <= v <= 2**31 - 1


@pytest.mark.parametrize("seed", [1, 2])
@pytest.mark.parametrize("n", [20, 100, 1000])
def test_render_scene_and_tree(oracle, small, seed, n):
    s = oracle.render_scene(seed, n)
    assert s.tobytes() == small[f"render_{n}_{seed}_pre"].tobytes()
    t = oracle.build(s)
    assert s.tobytes() == small[f"render_{n}_{seed}_post"].tobytes()   # in-place reorder (bvh.c:172-201)
    assert oracle.flatten(t).tobytes() == small[f"render_{n}_{seed}_tree"].tobytes()
    oracle.free(t)


def test_bench_scene_and_tree(oracle, small):
    s = oracle.bench_scene(1, 1000)
    assert s.tobytes() == small["bench_1000_1_pre"].tobytes()
    t = oracle.build(s, 0, 999, 20)                                     # benchmark.c:317
    assert s.tobytes() == small["bench_1000_1_post"].tobytes()
    assert oracle.flatten(t).tobytes() == small["bench_1000_1_tree"].tobytes()
    oracle.free(t)


@pytest.mark.parametrize("key", ["render_10000_1", "render_100000_1"])
def test_large_tree_hashes(oracle, golden, key):
    g = golden["scenes"][key]
    n = int(key.split("_")[1])
    s = oracle.render_scene(1, n)
    assert sha(s) == g["scene_sha"]
    t = oracle.build(s)
    flat = oracle.flatten(t)
    oracle.free(t)
    assert sha(s) == g["post_sha"]
    assert sha(flat) == g["tree_sha"]
    assert len(flat) == g["nodes"]
    assert int(((flat["skip"] & abi.NODE_EMPTY) != 0).sum()) == g["empty_leaves"]


def _hits_equal(a, b):
    return a.tobytes() == b.tobytes()


def test_closest_hits_render(oracle, small):
    s = small["render_1000_1_post"].copy()
    t = oracle.build(small["render_1000_1_pre"].copy())
    got = oracle.intersect(t, s, small["hits_rays"])
    oracle.free(t)
    assert _hits_equal(got, small["hits_render_1000"])


def test_closest_hits_bench(oracle, small):
    s = small["bench_1000_1_post"].copy()
    t = oracle.build(small["bench_1000_1_pre"].copy(), 0, 999, 20)
    got = oracle.intersect(t, s, small["hits_bench_rays"])
    oracle.free(t)
    assert _hits_equal(got, small["hits_bench_1000"])


def test_sphere_and_slab_primitives(oracle, small):
    rays = small["hits_rays"]
    got = oracle.sphere_pairs(rays, small["pairs_spheres"])
    ref = small["pairs_sphere_hits"]
    assert got.tobytes() == ref.tobytes()
    assert (oracle.aabb_pairs(rays, small["pairs_boxes"]) == small["pairs_box_hits"]).all()
    # empty boxes always pass (bvh.c:19-24 + hit.c:49-82)
    assert small["pairs_box_hits"][:64].all()


def test_trace_rays(oracle, small):
    s = small["render_1000_1_post"].copy()
    t = oracle.build(small["render_1000_1_pre"].copy())
    rays = small["hits_rays"]
    assert (oracle.trace_rays(rays, s, t, depth=1, mode=0, seed=3) == small["trace_d1_mode0"]).all()
    assert (oracle.trace_rays(rays, s, t, depth=5, mode=1, seed=3) == small["trace_d5_mode1"]).all()
    assert (oracle.trace_rays(rays[:1500], s, None, depth=5, use_bvh=False, mode=1, seed=3)
            == small["trace_d5_mode1_brute"]).all()
    oracle.free(t)


def test_camera_rays(oracle, golden, small):
    cams = [abi.Camera.from_numpy(c) for c in small["cameras"]]
    for key, g in golden["camera_rays"].items():
        res, ci = key.split("_cam")
        W, H = map(int, res.split("x"))
        got = oracle.camera_rays(cams[int(ci)], W, H, rows=g["rows"])
        assert got.tobytes() == small[f"camrays_{key}"].tobytes()
        assert sha(got) == g["sha"]


def _frame_cases(golden, max_pixels):
    out = []
    for key, g in golden["frames"].items():
        p = parse_frame_key(key)
        if p["W"] * g["rows"] <= max_pixels:
            out.append(key)
    return out


def test_frames(oracle, golden, small):
    cams = [abi.Camera.from_numpy(c) for c in small["cameras"]]
    done = 0
    for key in _frame_cases(golden, 2_100_000):
        p = parse_frame_key(key)
        if p["n"] >= 100000:
            continue  # the 100k / 1M scenes are covered by the GPU tests
        s = oracle.render_scene(1, p["n"]) if p["kind"] == "render" else oracle.bench_scene(1, p["n"])
        t = oracle.build(s)
        rows = np.arange(0, p["H"], p["step"], dtype=np.int32)
        # depth 1 never uses a draw (renderer.c:23-24), so the contract path
        # (thread-parallel) reproduces the glibc-stream frame
        mode = 1 if p["depth"] == 1 else p["mode"]
        img = oracle.render(cams[p["cam"]], p["W"], p["H"], s, t, depth=p["depth"], use_bvh=p["use_bvh"],
                            mode=mode, seed=p["seed"], rows=rows)
        oracle.free(t)
        assert sha(img) == golden["frames"][key]["sha"], key
        if "frame_" + key in small:
            assert (img == small["frame_" + key]).all()
        done += 1
    assert done >= 20


def test_accumulate_restatement(oracle):
    """main.c:368-370 / 394-401 (not linkable: main.c needs SDL) -- restated
    only, so checked for its defining properties: a fresh frame stores c/255,
    N identical accumulated frames show the colour again (up to the float
    sum's rounding), and frames=2 after one fresh frame halves it."""
    rng = np.random.default_rng(0)
    c = rng.integers(0, 256, (500, 4), dtype=np.uint8)
    acc = np.zeros(500 * 3, np.float32)
    shown = oracle.accumulate(c, acc, True, 1)
    assert (shown == c).all()
    assert np.allclose(acc.reshape(-1, 3), c[:, :3] / 255.0, atol=1e-7)
    shown2 = oracle.accumulate(c, acc, False, 2)
    assert (np.abs(shown2[:, :3].astype(int) - c[:, :3]) <= 1).all()
    acc0 = np.zeros(500 * 3, np.float32)
    half = oracle.accumulate(c, acc0, False, 2)   # main.c first frame: camera.move == 0 -> frames = 2
    assert (np.abs(half[:, :3].astype(int) - c[:, :3] // 2) <= 1).all()


def test_oracle_flat_dfs_equals_pointer_dfs(mirt, oracle, small):
    """o_intersect_flat (hit.c:91-109 over a flat tree, used for the 10M /
    100M benchmark-mode points) equals o_intersect on the oracle's own
    pointer tree, on the render and the benchmark.c:317-style build."""
    for kind, start_end_depth in (("render", (0, None, 0)), ("bench", (0, 999, 20))):
        pre = small[f"{kind}_1000_1_pre"]
        so = pre.copy()
        st, en, d = start_end_depth
        t = oracle.build(so, st, en, d)
        s = pre.copy()
        flat = mirt.build_bvh(s, st, en, d)
        rays = small["hits_rays"] if kind == "render" else small["hits_bench_rays"]
        ns = len(s) if en is None else en
        want = oracle.intersect(t, so[:ns], rays)
        oracle.free(t)
        got = oracle.intersect_flat(flat.nodes, s[:ns], rays)
        assert got.tobytes() == want.tobytes(), kind
        assert int(want["hit"].sum()) > (50 if kind == "render" else 0), kind
