"""GPU parity: the HIP path (libmirt.so on cuda:0, called through the C ABI)
against the reference's golden vectors and the oracle. Bit-exact: every
test compares bytes (the 1e-5 per-channel float tolerance of BASELINE.json's
north_star reduces to an exact u8 match)."""
import numpy as np
import pytest

from conftest import parse_frame_key, sha

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def scene1000(mirt, small):
    s = small["render_1000_1_pre"].copy()
    b = mirt.build_bvh(s)
    return s, b


def cams(mirt, small):
    return [mirt.abi.Camera.from_numpy(c) for c in small["cameras"]]


def test_camera_rays(gpu, mirt, golden, small):
    cs = cams(mirt, small)
    for key, g in golden["camera_rays"].items():
        res, ci = key.split("_cam")
        W, H = map(int, res.split("x"))
        rays = gpu.get_camera_rays(cs[int(ci)], W, H)
        got = rays[g["rows"]]
        assert got.tobytes() == small[f"camrays_{key}"].tobytes(), key


def test_sphere_pairs(gpu, small):
    got = gpu.ray_sphere_intersect(small["hits_rays"], small["pairs_spheres"])
    assert got.tobytes() == small["pairs_sphere_hits"].tobytes()


def test_aabb_pairs(gpu, small):
    got = gpu.ray_aabb_intersect(small["hits_rays"], small["pairs_boxes"])
    assert (got == small["pairs_box_hits"]).all()


def test_closest_hits_bvh(gpu, mirt, small, scene1000):
    s, b = scene1000
    gpu.upload(s, b)
    got = gpu.ray_bvh_intersect(small["hits_rays"])
    assert got.tobytes() == small["hits_render_1000"].tobytes()


def test_closest_hits_bench_tree(gpu, mirt, small):
    s = small["bench_1000_1_pre"].copy()
    b = mirt.build_bvh(s, 0, 999, 20)
    gpu.upload(s, b)
    got = gpu.ray_bvh_intersect(small["hits_bench_rays"])
    assert got.tobytes() == small["hits_bench_1000"].tobytes()


def test_closest_hits_brute(gpu, oracle, small, scene1000):
    s, b = scene1000
    gpu.upload(s, b)
    rays = small["hits_rays"]
    got = gpu.closest_hit(rays, use_bvh=False)
    ref = oracle.intersect(None, s, rays, use_bvh=False)
    assert got.tobytes() == ref.tobytes()


def test_trace_rays(gpu, small, scene1000):
    s, b = scene1000
    gpu.upload(s, b)
    rays = small["hits_rays"]
    assert (gpu.trace_ray(rays, depth=1, seed=3) == small["trace_d1_mode0"]).all()
    assert (gpu.trace_ray(rays, depth=5, seed=3) == small["trace_d5_mode1"]).all()
    assert (gpu.trace_ray(rays[:1500], depth=5, use_bvh=False, seed=3) == small["trace_d5_mode1_brute"]).all()


def test_pointer_tree_upload(gpu, mirt, small):
    """mirt_scene_upload flattens a caller's pointer tree (drop-in path)."""
    s = small["render_1000_1_pre"].copy()
    root = mirt.build_bvh_node(s)
    gpu.upload(s, root)
    mirt.free_bvh(root)
    got = gpu.ray_bvh_intersect(small["hits_rays"])
    assert got.tobytes() == small["hits_render_1000"].tobytes()


_scene_cache = {}


def _scene(mirt, kind, n):
    if (kind, n) not in _scene_cache:
        s = mirt.create_random_spheres(n, 1) if kind == "render" else mirt.create_benchmark_spheres(n, 1)
        b = mirt.build_bvh(s)
        _scene_cache.clear()
        _scene_cache[(kind, n)] = (s, b)
    return _scene_cache[(kind, n)]


def test_golden_frames(gpu, mirt, golden, small):
    """Every golden framebuffer: 160x90 .. 1920x1080, 100 .. 1M spheres,
    depth 1 (the unmodified reference's glibc stream: draws unused) and depth
    5 (per-pixel contract), BVH and brute force, two cameras."""
    cs = cams(mirt, small)
    keys = sorted(golden["frames"], key=lambda k: (parse_frame_key(k)["kind"], parse_frame_key(k)["n"]))
    for key in keys:
        p = parse_frame_key(key)
        if p["mode"] == 0 and p["depth"] > 1:
            continue  # glibc serial stream: not reproducible in parallel by design
        s, b = _scene(mirt, p["kind"], p["n"])
        gpu.upload(s, b)
        img = gpu.render_frame(cs[p["cam"]], p["W"], p["H"], depth=p["depth"], use_bvh=p["use_bvh"],
                               seed=p["seed"])
        img = img[::p["step"]]
        assert sha(img) == golden["frames"][key]["sha"], key
        if "frame_" + key in small:
            assert (img == small["frame_" + key]).all(), key


@pytest.mark.parametrize("world", [2, 3, 8])
def test_sharded_frames_identical(gpu, mirt, world):
    """Row-block shards reassembled == the one-shard frame (1080p, 10k)."""
    from importlib import import_module
    shard = import_module("cs201_sah-bvh_ray_tracer_amd.shard")
    import torch
    s, b = _scene(mirt, "render", 10000)
    gpu.upload(s, b)
    cam = mirt.default_camera()
    full = gpu.render_frame(cam, 1920, 1080, depth=5, seed=1)
    slabs = [gpu.render_frame(cam, 1920, 1080, depth=5, seed=1, shard=r, num_shards=world)[None]
             for r in range(world)]
    frame = shard.assemble_gather(slabs, 1080, 8)[0]
    assert (frame == full).all()
    assert (shard.assemble_direct(slabs, 1080, 8)[0] == full).all()


def test_accumulate_matches_oracle(gpu, mirt, oracle, small):
    """main.c:379-408: 3 accumulated samples after a fresh frame."""
    s, b = _scene(mirt, "render", 1000)
    gpu.upload(s, b)
    cam = mirt.default_camera()
    W, H = 160, 90
    t = oracle.build(small["render_1000_1_pre"].copy())
    acc = np.zeros(W * H * 3, np.float32)
    for k in range(4):
        got = gpu.render_frame(cam, W, H, depth=5, seed=4, sample=k, accumulate=k > 0, frames=k + 1)
        col = oracle.render(cam, W, H, s, t, depth=5, mode=1, seed=4, sample=k)
        ref = oracle.accumulate(col, acc, k == 0, k + 1).reshape(H, W, 4)
        assert (got == ref).all(), k
    assert gpu.accum(W * H * 3).tobytes() == acc.tobytes()
    oracle.free(t)


@pytest.mark.parametrize("depth,trav", [(5, 5), (1, 5), (5, 0)])
def test_frames_in_flight_match_successive_frames(gpu, mirt, oracle, small, depth, trav):
    """samples = 4 in one launch == 4 successive calls of the accumulating
    loop (main.c:379-408): same display, same accumulation buffer; checked
    against the oracle too, on a whole frame and on shard 1 of 3."""
    s, b = _scene(mirt, "render", 1000)
    gpu.upload(s, b)
    cam = mirt.default_camera()
    W, H = 160, 90
    t = oracle.build(small["render_1000_1_pre"].copy())
    old = gpu.get_option(mirt.abi.OPT_TRAVERSAL)
    try:
        gpu.set_option(mirt.abi.OPT_TRAVERSAL, trav)
        for shard, world in ((0, 1), (1, 3)):
            seq = None
            for k in range(4):
                seq = gpu.render_frame(cam, W, H, depth=depth, seed=4, sample=k, accumulate=k > 0, frames=k + 1,
                                       shard=shard, num_shards=world)
            acc_seq = gpu.accum(seq.shape[0] * W * 3)
            one = gpu.render_frame(cam, W, H, depth=depth, seed=4, sample=0, samples=4, shard=shard,
                                   num_shards=world)
            assert (one == seq).all(), shard
            assert gpu.accum(seq.shape[0] * W * 3).tobytes() == acc_seq.tobytes()
            # continuing an accumulation: frames 4..6 after the 4 above
            more = gpu.render_frame(cam, W, H, depth=depth, seed=4, sample=4, samples=3, accumulate=True, frames=5,
                                    shard=shard, num_shards=world)
            acc = np.zeros(W * H * 3, np.float32)
            for k in range(7):
                col = oracle.render(cam, W, H, s, t, depth=depth, mode=1, seed=4, sample=k)
                ref = oracle.accumulate(col, acc, k == 0, k + 1).reshape(H, W, 4)
            rows = mirt.shard_rows(mirt.frame_desc(W, H, shard=shard, num_shards=world))
            assert (more == ref[rows]).all(), shard
    finally:
        gpu.set_option(mirt.abi.OPT_TRAVERSAL, old)
        oracle.free(t)


def test_frames_in_flight_raw_slabs(gpu, mirt):
    """Without an accumulation buffer a launch of samples = 3 leaves frame j
    (RNG sample j) in slab j: each equals the fresh single frame."""
    import torch
    s, b = _scene(mirt, "render", 10000)
    gpu.upload(s, b)
    cam = mirt.default_camera()
    W, H = 320, 180
    fd = mirt.frame_desc(W, H, depth=5, seed=2, sample=5, samples=3)
    out = torch.zeros((3, H, W), dtype=torch.int32, device="cuda")
    gpu.render_frame_device(cam, fd, out.data_ptr(), None, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint8).reshape(3, H, W, 4)
    for j in range(3):
        ref = gpu.render_frame(cam, W, H, depth=5, seed=2, sample=5 + j)
        assert (got[j] == ref).all(), j


@pytest.mark.parametrize("world", [2, 4, 8])
def test_weak_scaling_step_identical(gpu, mirt, world):
    """The bench's weak-scaling step at N ranks (N frames in flight, rows
    interleaved over N shards, display slabs gathered) shows the same bytes
    as the same N frames accumulated on one GPU."""
    from importlib import import_module
    import torch
    shard = import_module("cs201_sah-bvh_ray_tracer_amd.shard")
    s, b = _scene(mirt, "render", 10000)
    gpu.upload(s, b)
    cam = mirt.default_camera()
    W, H = 1920, 1080
    full = gpu.render_frame(cam, W, H, depth=5, seed=1, samples=world)
    slabs = [gpu.render_frame(cam, W, H, depth=5, seed=1, samples=world, shard=r, num_shards=world)[None]
             for r in range(world)]
    frame = shard.assemble_gather(slabs, H, 8)[0]
    assert (frame == full).all()


def test_double_buffered_frames_identical(gpu, mirt):
    """Launches in flight (mirt_multi, two lanes of contexts alternating
    frames on their own streams, launches overlapping) leave every frame's
    bytes unchanged."""
    s, b = _scene(mirt, "render", 10000)
    gpu.upload(s, b)
    cam = mirt.default_camera()
    W, H = 640, 360
    bufs = [mirt.HostBuffer((H, W, 4)) for _ in range(5)]
    try:
        with mirt.MultiRenderer([0], lanes=2) as m:
            m.upload(s, b)
            for k in range(5):
                m.render_frames_async(cam, mirt.frame_desc(W, H, depth=5, seed=3, sample=k), [bufs[k]])
                if k % 2 == 1:
                    m.wait()
            m.wait()
            got = [x.array.copy() for x in bufs]
    finally:
        for x in bufs:
            x.close()
    for k in range(5):
        ref = gpu.render_frame(cam, W, H, depth=5, seed=3, sample=k)
        assert (got[k] == ref).all(), k


def test_async_host_frames_pipelined(gpu, mirt, golden):
    """bench.py's host-inclusive loop: three ctxs take successive frames,
    each frame's kernels and its D2H copy into page-locked memory enqueued
    with mirt_render_frame_async; every frame that lands on the host equals
    the blocking call's (and frame 0 the reference's golden 1080p frame)."""
    s, b = _scene(mirt, "render", 10000)
    gpu.upload(s, b)
    extra = [mirt.Renderer(0), mirt.Renderer(0)]
    rs = [gpu] + extra
    bufs = [mirt.HostBuffer((1080, 1920, 4)) for _ in rs]
    try:
        for x in extra:
            x.upload(s, b)
        cam = mirt.default_camera()
        got = []
        for k in range(7):
            i = k % 3
            rs[i].wait()
            if k >= 3:
                got.append(bufs[i].array.copy())
            rs[i].render_frame_async(cam, mirt.frame_desc(1920, 1080, depth=5, seed=1, sample=k), bufs[i])
        for x in rs:
            x.wait()
        for k in range(4, 7):
            got.append(bufs[k % 3].array.copy())
        assert len(got) == 7
        assert sha(got[0]) == golden["frames"]["1920x1080_render10000_d5_m1_b1_s1_c0_step1"]["sha"]
        for k in (1, 6):
            assert (got[k] == gpu.render_frame(cam, 1920, 1080, depth=5, seed=1, sample=k)).all(), k
        with pytest.raises(mirt.MirtError):
            gpu.render_frame_async(cam, mirt.frame_desc(1920, 1080), np.zeros(16, np.uint8))
    finally:
        for x in bufs:
            x.close()
        for x in extra:
            x.close()


@pytest.mark.parametrize("W,H,n", [(160, 90, 1000), (1920, 1080, 10000)])
def test_shared_accumulation_frames_in_flight(gpu, mirt, oracle, small, W, H, n):
    """main.c:379-408 with frames in flight (INTEGRATION.md's interactive
    recipe): four ctxs sharing ONE accumulation buffer (mirt_ctx_share_accum)
    take successive frames of the still-camera loop with
    mirt_render_frame_async, frame k waiting only for frame k - 4 on the
    same ctx. Every host frame equals frame k of 8 successive blocking
    mirt_render_frame calls on one ctx (and, at 160x90, the oracle's
    accumulation, o_accumulate); the shared buffer equals the oracle's."""
    s, b = _scene(mirt, "render", n)
    cam = mirt.default_camera()
    rs = [mirt.Renderer(0) for _ in range(4)]
    bufs = [mirt.HostBuffer((H, W, 4)) for _ in rs]
    try:
        for x in rs:
            x.upload(s, b)
            x.share_accum(rs[0])
            x.set_option(mirt.abi.OPT_BOUNCE_BLOCKS, 384)
        got = [None] * 8
        for k in range(8):
            i = k % 4
            rs[i].wait()
            if k >= 4:
                got[k - 4] = bufs[i].array.copy()
            fd = mirt.frame_desc(W, H, depth=5, seed=4, sample=k, accumulate=k > 0, frames=k + 1)
            rs[i].render_frame_async(cam, fd, bufs[i])
        for k in range(4, 8):
            rs[k % 4].wait()
            got[k] = bufs[k % 4].array.copy()
        acc_shared = rs[1].accum(W * H * 3)
        gpu.upload(s, b)
        for k in range(8):
            seq = gpu.render_frame(cam, W, H, depth=5, seed=4, sample=k, accumulate=k > 0, frames=k + 1)
            assert (got[k] == seq).all(), k
        assert acc_shared.tobytes() == gpu.accum(W * H * 3).tobytes()
        seq_fresh = [gpu.render_frame(cam, W, H, depth=5, seed=4, sample=k) for k in range(8)]
        if n <= 1000:
            t = oracle.build(small["render_1000_1_pre"].copy())
            acc = np.zeros(W * H * 3, np.float32)
            for k in range(8):
                col = oracle.render(cam, W, H, s, t, depth=5, mode=1, seed=4, sample=k)
                ref = oracle.accumulate(col, acc, k == 0, k + 1).reshape(H, W, 4)
                assert (got[k] == ref).all(), k
            oracle.free(t)
            assert acc_shared.tobytes() == acc.tobytes()
        # detached again: a private buffer
        rs[1].share_accum(None)
        with pytest.raises(mirt.MirtError):
            rs[1].accum(W * H * 3)
        # frames in flight written in place (MIRT_OPT_ZERO_COPY 2) into the
        # page-locked buffers: the same frames (private buffers again first)
        for x in rs:
            x.share_accum(None)
            x.set_option(mirt.abi.OPT_ZERO_COPY, 2)
        for k in range(8):
            i = k % 4
            rs[i].wait()
            if k >= 4:
                assert (bufs[i].array == seq_fresh[k - 4]).all(), k - 4
            fd = mirt.frame_desc(W, H, depth=5, seed=4, sample=k)
            rs[i].render_frame_async(cam, fd, bufs[i])
        for k in range(4, 8):
            rs[k % 4].wait()
            assert (bufs[k % 4].array == seq_fresh[k]).all(), k
        for x in rs:
            x.set_option(mirt.abi.OPT_ZERO_COPY, 1)
    finally:
        for x in bufs:
            x.close()
        for x in rs:
            x.close()


def test_lazy_fold_fresh_frames_in_flight(gpu, mirt):
    """The lazy fold: fresh frames on four ctxs sharing one accumulation
    buffer leave their displays pending instead of folding in order. After
    six fresh frames in flight the shared buffer (read back) is the last
    frame's colours / 255; an accumulating frame on ANOTHER ctx then continues
    from it; a fresh frame on the pending frame's OWN ctx supersedes it; and
    the frames shown equal one ctx's blocking sequence throughout."""
    W, H = 320, 180
    s, b = _scene(mirt, "render", 10000)
    cam = mirt.default_camera()
    rs = [mirt.Renderer(0) for _ in range(4)]
    bufs = [mirt.HostBuffer((H, W, 4)) for _ in rs]
    try:
        for x in rs:
            x.upload(s, b)
            x.share_accum(rs[0])
        seq = [(k, False, 1) for k in range(7)] + [(7, True, 2), (8, True, 3), (9, False, 1), (10, True, 2)]
        # frame 6 supersedes frame 5 on the same ctx; frame 7 (another ctx) takes frame 6's pending
        # display from ctx 1's slab; frame 8 then writes that slab (its guard); frame 10 accumulates
        # on the ctx whose own slab holds the pending frame 9
        ctx_of = [0, 1, 2, 3, 0, 1, 1, 3, 1, 0, 0]
        got = []
        for j, (k, acc, fr) in enumerate(seq):
            i = ctx_of[j]
            rs[i].wait()
            fd = mirt.frame_desc(W, H, depth=5, seed=9, sample=k, accumulate=acc, frames=fr)
            rs[i].render_frame_async(cam, fd, bufs[i])
            rs[i].wait()
            got.append(bufs[i].array.copy())
            if j == 5:
                shared_after_fresh = rs[2].accum(W * H * 3)
        gpu.upload(s, b)
        for j, (k, acc, fr) in enumerate(seq):
            want = gpu.render_frame(cam, W, H, depth=5, seed=9, sample=k, accumulate=acc, frames=fr)
            assert (got[j] == want).all(), j
            if j == 5:
                assert shared_after_fresh.tobytes() == gpu.accum(W * H * 3).tobytes()
        assert rs[3].accum(W * H * 3).tobytes() == gpu.accum(W * H * 3).tobytes()
    finally:
        for x in bufs:
            x.close()
        for x in rs:
            x.close()


def test_lazy_fold_many_in_flight(gpu, mirt):
    """Fresh frames issued on four sharing ctxs WITHOUT waiting between them
    (each ctx waits only for its own previous frame), then one accumulating
    frame: it must continue from the LAST fresh frame issued, whichever ctx
    finished last."""
    W, H = 640, 360
    s, b = _scene(mirt, "render", 10000)
    cam = mirt.default_camera()
    rs = [mirt.Renderer(0) for _ in range(4)]
    bufs = [mirt.HostBuffer((H, W, 4)) for _ in rs]
    try:
        for x in rs:
            x.upload(s, b)
            x.share_accum(rs[0])
        for k in range(9):
            i = k % 4
            rs[i].wait()
            rs[i].render_frame_async(cam, mirt.frame_desc(W, H, depth=5, seed=2, sample=k), bufs[i])
        i = 9 % 4
        rs[i].wait()
        rs[i].render_frame_async(cam, mirt.frame_desc(W, H, depth=5, seed=2, sample=9, accumulate=True, frames=2),
                                 bufs[i])
        for x in rs:
            x.wait()
        got = bufs[i].array.copy()
        gpu.upload(s, b)
        gpu.render_frame(cam, W, H, depth=5, seed=2, sample=8)
        want = gpu.render_frame(cam, W, H, depth=5, seed=2, sample=9, accumulate=True, frames=2)
        assert (got == want).all()
    finally:
        for x in bufs:
            x.close()
        for x in rs:
            x.close()


def test_share_after_private_async_frames(gpu, mirt):
    """A ctx that starts sharing a buffer whose owner still has frames in
    flight that wrote it privately (no fold event): the sharer's first fold
    must follow them. Owner: three async accumulating frames, no
    wait; then the share and the sharer's frame 4: equals four blocking
    frames on one ctx."""
    W, H = 640, 360
    s, b = _scene(mirt, "render", 10000)
    cam = mirt.default_camera()
    rs = [mirt.Renderer(0) for _ in range(2)]
    bufs = [mirt.HostBuffer((H, W, 4)) for _ in rs]
    try:
        for x in rs:
            x.upload(s, b)
        for k in range(3):
            fd = mirt.frame_desc(W, H, depth=5, seed=4, sample=k, accumulate=k > 0, frames=k + 1)
            rs[0].render_frame_async(cam, fd, bufs[0])
        rs[1].share_accum(rs[0])
        fd = mirt.frame_desc(W, H, depth=5, seed=4, sample=3, accumulate=True, frames=4)
        rs[1].render_frame_async(cam, fd, bufs[1])
        rs[1].wait()
        rs[0].wait()
        got = bufs[1].array.copy()
        gpu.upload(s, b)
        for k in range(4):
            seq = gpu.render_frame(cam, W, H, depth=5, seed=4, sample=k, accumulate=k > 0, frames=k + 1)
        assert (got == seq).all()
    finally:
        for x in bufs:
            x.close()
        for x in rs:
            x.close()


def test_counts_match_oracle(gpu, mirt, oracle):
    s, b = _scene(mirt, "render", 10000)
    gpu.upload(s, b)
    cam = mirt.default_camera()
    s2 = mirt.create_random_spheres(10000, 1)
    t = oracle.build(s2)
    _, cnt = oracle.render(cam, 320, 180, s2, t, depth=5, mode=1, seed=1, counts=True)
    oracle.free(t)
    gpu.set_option(mirt.abi.OPT_PRUNE, 0)        # the reference's exhaustive DFS
    try:
        got = gpu.count_frame(cam, 320, 180, depth=5, seed=1)
        d1 = gpu.count_frame(cam, 320, 180, depth=1, seed=1)
    finally:
        gpu.set_option(mirt.abi.OPT_PRUNE, 1)
    assert (got["rays"], got["nodes"], got["spheres"]) == tuple(int(x) for x in cnt)
    # the camera-ray level of a depth-5 frame is the whole of a depth-1 frame
    assert (got["nodes_primary"], got["spheres_primary"], got["hits_primary"]) == \
        (d1["nodes"], d1["spheres"], d1["hits"])
    assert d1["nodes_primary"] == d1["nodes"]
    # pruning: same rays and hits, strictly less walking
    pr = gpu.count_frame(cam, 320, 180, depth=5, seed=1)
    assert (pr["rays"], pr["hits"], pr["hits_primary"]) == (got["rays"], got["hits"], got["hits_primary"])
    assert pr["nodes"] < got["nodes"] and pr["spheres"] < got["spheres"]


def _hard_rays(rng, spheres, n):
    """Rays that stress the pruning bound: bounce-like rays leaving sphere
    surfaces, rays grazing sphere silhouettes, and rays from anywhere."""
    from importlib import import_module
    abi = import_module("cs201_sah-bvh_ray_tracer_amd").abi
    c = spheres["center"].astype(np.float64)
    r = spheres["radius"].astype(np.float64)
    k = n // 3
    rays = np.zeros(3 * k, abi.RAY)
    # 1) leave a surface point into the outer hemisphere
    i = rng.integers(0, len(spheres), k)
    nrm = rng.normal(size=(k, 3))
    nrm /= np.linalg.norm(nrm, axis=1)[:, None]
    d = rng.normal(size=(k, 3))
    d /= np.linalg.norm(d, axis=1)[:, None]
    d *= np.sign((d * nrm).sum(1))[:, None]
    rays["origin"][:k] = c[i] + nrm * r[i][:, None]
    rays["direction"][:k] = d
    # 2) aim at a point within 0.1% of a sphere's silhouette
    i = rng.integers(0, len(spheres), k)
    lo, hi = c.min(0) - 10, c.max(0) + 10
    o = rng.uniform(lo, hi, (k, 3))
    u = rng.normal(size=(k, 3))
    u /= np.linalg.norm(u, axis=1)[:, None]
    tgt = c[i] + u * (r[i] * rng.uniform(0.999, 1.001, k))[:, None]
    d = tgt - o
    d /= np.linalg.norm(d, axis=1)[:, None]
    rays["origin"][k:2 * k] = o
    rays["direction"][k:2 * k] = d
    # 3) anywhere, any direction
    d = rng.normal(size=(k, 3))
    d /= np.linalg.norm(d, axis=1)[:, None]
    rays["origin"][2 * k:] = rng.uniform(lo, hi, (k, 3))
    rays["direction"][2 * k:] = d
    return rays


@pytest.mark.parametrize("kind,n", [("render", 10000), ("bench", 100000)])
def test_pruning_keeps_every_hit(gpu, mirt, oracle, kind, n):
    """Closest hits with pruning == without == the oracle's reference DFS,
    bit for bit, on 300k hard rays (oracle on a 30k subset)."""
    abi = mirt.abi
    s, b = _scene(mirt, kind, n)
    gpu.upload(s, b)
    rays = _hard_rays(np.random.default_rng(7), s, 300_000)
    try:
        gpu.set_option(abi.OPT_PRUNE, 1)
        on = gpu.ray_bvh_intersect(rays)                  # ordered packet walk
        gpu.set_option(abi.OPT_ORDERED, 0)
        dfs = gpu.ray_bvh_intersect(rays)                 # pruned, DFS order
        gpu.set_option(abi.OPT_PRUNE, 0)
        off = gpu.ray_bvh_intersect(rays)                 # the reference's walk
    finally:
        gpu.set_option(abi.OPT_PRUNE, 1)
        gpu.set_option(abi.OPT_ORDERED, 1)
    assert on.tobytes() == off.tobytes()
    assert dfs.tobytes() == off.tobytes()
    assert (on["hit"] == 1).sum() > 50_000
    s2 = mirt.create_random_spheres(n, 1) if kind == "render" else mirt.create_benchmark_spheres(n, 1)
    t = oracle.build(s2)
    sub = np.ascontiguousarray(rays[::10])
    ref = oracle.intersect(t, s2, sub)
    oracle.free(t)
    assert on[::10].tobytes() == ref.tobytes()


def test_phase_timing(gpu, mirt):
    s, b = _scene(mirt, "render", 10000)
    gpu.upload(s, b)
    cam = mirt.default_camera()
    gpu.render_frame(cam, 320, 180, depth=5, seed=1)
    primary, bounce = gpu.last_phase_ms()
    assert primary > 0 and bounce > 0
    gpu.render_frame(cam, 320, 180, depth=1, seed=1)   # depth 1 has no bounce pass
    with pytest.raises(mirt.MirtError):
        gpu.last_phase_ms()


def test_sentinel_and_edge_scenes(gpu, mirt, oracle):
    abi = mirt.abi
    # a hand-made tree whose right leaf is the &spheres[N] sentinel
    s = np.zeros(1, abi.SPHERE)
    s["center"] = [0, 0, 0]
    s["radius"] = 5
    s["color"] = [10, 20, 30, 255]
    nodes = np.zeros(3, abi.NODE)
    nodes[0] = ([-5, -5, -5], [5, 5, 5], -1, 3)
    nodes[1] = ([-5, -5, -5], [5, 5, 5], 0, 2)
    nodes[2] = ([np.inf] * 3, [-np.inf] * 3, 1, 3 | abi.NODE_EMPTY)
    gpu.upload(s, mirt.Bvh(nodes))
    rays = np.zeros(2, abi.RAY)
    rays["origin"] = [[0, 0, 20], [7, 0, 20]]
    rays["direction"] = [[0, 0, -1], [0, 0, -1]]
    h = gpu.ray_bvh_intersect(rays)
    assert h["hit"].tolist() == [1, 0] and h["sphere"].tolist() == [0, -1]
    assert h["t"][0] == np.float32(15.0)
    # empty scene: every pixel is sky, brute force and an empty tree alike
    gpu.upload(np.zeros(0, abi.SPHERE), None)
    cam = mirt.default_camera()
    img = gpu.render_frame(cam, 64, 32, depth=5, use_bvh=False)
    s0 = np.zeros(0, abi.SPHERE)
    ref = oracle.render(cam, 64, 32, s0, None, depth=5, use_bvh=False, mode=1)
    assert (img == ref).all()


@pytest.mark.parametrize("trav", [0, 5])
@pytest.mark.parametrize("fast,prune,ordered", [(0, 0, 0), (1, 0, 0), (1, 1, 0), (1, 1, 1)])
@pytest.mark.parametrize("defer", [0, 1])
def test_all_schedules_bit_identical(gpu, mirt, golden, small, scene1000, trav, fast, prune, ordered, defer):
    """Every traversal schedule x slab-test form x pruning gives the
    reference's bytes: per-ray hits and traces, and the 1080p 10k
    depth-1/depth-5 frames."""
    abi = mirt.abi
    gpu.set_option(abi.OPT_TRAVERSAL, trav)
    gpu.set_option(abi.OPT_FAST_SLAB, fast)
    gpu.set_option(abi.OPT_PRUNE, prune)
    gpu.set_option(abi.OPT_ORDERED, ordered)
    gpu.set_option(abi.OPT_DEFER, defer)
    try:
        s, b = scene1000
        gpu.upload(s, b)
        assert gpu.ray_bvh_intersect(small["hits_rays"]).tobytes() == small["hits_render_1000"].tobytes()
        assert (gpu.trace_ray(small["hits_rays"], depth=5, seed=3) == small["trace_d5_mode1"]).all()
        s10, b10 = _scene(mirt, "render", 10000)
        gpu.upload(s10, b10)
        cam = mirt.default_camera()
        for depth, mode in [(1, 0), (5, 1)]:
            key = f"1920x1080_render10000_d{depth}_m{mode}_b1_s1_c0_step1"
            img = gpu.render_frame(cam, 1920, 1080, depth=depth, seed=1)
            assert sha(img) == golden["frames"][key]["sha"], key
    finally:
        gpu.set_option(abi.OPT_TRAVERSAL, abi.TRAV_WAVEFRONT)
        gpu.set_option(abi.OPT_FAST_SLAB, 1)
        gpu.set_option(abi.OPT_PRUNE, 1)
        gpu.set_option(abi.OPT_ORDERED, 1)
        gpu.set_option(abi.OPT_DEFER, 1)


def test_errors_are_loud(gpu, mirt):
    cam = mirt.default_camera()
    gpu.upload(np.zeros(0, mirt.abi.SPHERE), None)
    with pytest.raises(mirt.MirtError):
        gpu.render_frame(cam, 64, 32, depth=5, use_bvh=True)   # no tree uploaded
    with pytest.raises(mirt.MirtError):
        gpu.render_frame(cam, 64, 32, depth=9)                  # depth above the register budget
    bad = np.zeros(2, mirt.abi.NODE)
    bad[0] = ([0] * 3, [1] * 3, -1, 7)                          # skip out of range
    with pytest.raises(mirt.MirtError):
        gpu.upload(np.zeros(1, mirt.abi.SPHERE), mirt.Bvh(bad))


def test_ties_go_to_the_later_leaf(gpu, mirt, oracle):
    """Duplicate spheres tie exactly on t; hit.c:108 keeps the later DFS leaf.
    The ordered walk (nearer child first) must pick the same one."""
    abi = mirt.abi
    base = mirt.create_random_spheres(2000, 5)
    dup = base[:600].copy()
    dup["color"][:, 0] ^= 0x55                    # tell the copies apart
    s = np.concatenate([base, dup])
    s2 = s.copy()
    b = mirt.build_bvh(s)
    gpu.upload(s, b)
    rays = _hard_rays(np.random.default_rng(11), s, 60_000)
    try:
        on = gpu.ray_bvh_intersect(rays)
        gpu.set_option(abi.OPT_PRUNE, 0)
        off = gpu.ray_bvh_intersect(rays)
    finally:
        gpu.set_option(abi.OPT_PRUNE, 1)
    t = oracle.build(s2)
    ref = oracle.intersect(t, s2, rays)
    oracle.free(t)
    assert on.tobytes() == ref.tobytes()
    assert off.tobytes() == ref.tobytes()
    hit = on["hit"] == 1
    assert hit.sum() > 10_000


def test_one_sided_chains_frame(gpu, mirt, oracle):
    """Spheres sharing one centre send bvh.c's SAH (bvh.c:139-170) into its
    fallback: every plane leaves a side empty, so the split lands at x = 0 and
    one child is a 0-sphere leaf -- a chain of one-sided nodes down to the
    depth-40 cap, whose leaf tests only its first sphere. The derived walk
    layouts skip such chains (render.hip live_node) and fill four-wide nodes
    greedily; the frame, per-ray hits and traces must stay the reference's."""
    abi = mirt.abi
    base = mirt.create_random_spheres(3000, 7)
    cl = np.repeat(base[:40], 6)                   # 40 clusters of 6 coincident spheres
    cl["color"][:, 2] ^= (np.arange(len(cl)) % 6 * 37).astype(np.uint8)
    s = np.concatenate([base, cl])
    s2 = s.copy()
    b = mirt.build_bvh(s)
    flat = b.nodes
    leaf = flat["sphere"] >= 0
    empty = (flat["skip"] & abi.NODE_EMPTY) != 0
    assert (leaf & empty).sum() > 1000             # long fallback chains are present
    gpu.upload(s, b)
    cam = mirt.default_camera()
    img = gpu.render_frame(cam, 320, 180, depth=5, seed=1)
    t = oracle.build(s2)
    ref = oracle.render(cam, 320, 180, s2, t, depth=5, use_bvh=True, mode=1, seed=1)
    rays = _hard_rays(np.random.default_rng(5), s2, 30_000)
    hits = oracle.intersect(t, s2, rays)
    oracle.free(t)
    assert (img == ref).all(), int((img != ref).any(-1).sum())
    assert gpu.ray_bvh_intersect(rays).tobytes() == hits.tobytes()


def test_ordered_walk_stays_within_its_lanes(gpu, mirt):
    """The ordered packet walk may only carry lanes that passed every box on
    the path. A lane-mask leak lets inactive lanes (e.g. the deferred
    zero-component rays of the centre row) walk the whole tree without
    changing any result, so parity cannot see it; per-wave loop steps can:
    no wave of the ordered walk may take more steps than the slowest wave
    of the DFS-order walk."""
    abi = mirt.abi
    s, b = _scene(mirt, "render", 10000)
    gpu.upload(s, b)
    cam = mirt.default_camera()
    gpu.set_option(abi.OPT_TRAVERSAL, abi.TRAV_TILE)
    try:
        gpu.set_option(abi.OPT_ORDERED, 0)
        dfs = gpu.wave_stats(cam, 1920, 1080, depth=1)
        gpu.set_option(abi.OPT_ORDERED, 1)
        ordered = gpu.wave_stats(cam, 1920, 1080, depth=1)
    finally:
        gpu.set_option(abi.OPT_TRAVERSAL, abi.TRAV_WAVEFRONT)
        gpu.set_option(abi.OPT_ORDERED, 1)
    assert ordered[:, 1].max() <= dfs[:, 1].max()
    assert ordered[:, 1].sum() < dfs[:, 1].sum()


@pytest.mark.parametrize("drain", [0, 1])
@pytest.mark.parametrize("threshold,blocks", [(40, 0), (8, 0), (56, 64), (20, 384)])
def test_bounce_modes_identical(gpu, mirt, golden, drain, threshold, blocks):
    """The bounce pass's modes (one ray per lane, with or without the quad
    drain), refill thresholds and grid sizes (384: the bench's grid with
    frames in flight) give the golden 1080p frame."""
    abi = mirt.abi
    s, b = _scene(mirt, "render", 10000)
    gpu.upload(s, b)
    cam = mirt.default_camera()
    try:
        gpu.set_option(abi.OPT_QUAD_DRAIN, drain)
        gpu.set_option(abi.OPT_BOUNCE_THRESHOLD, threshold)
        gpu.set_option(abi.OPT_BOUNCE_BLOCKS, blocks)
        img = gpu.render_frame(cam, 1920, 1080, depth=5, seed=1)
    finally:
        gpu.set_option(abi.OPT_QUAD_DRAIN, 1)
        gpu.set_option(abi.OPT_BOUNCE_THRESHOLD, 20)   # the library default
        gpu.set_option(abi.OPT_BOUNCE_BLOCKS, 0)
    key = "1920x1080_render10000_d5_m1_b1_s1_c0_step1"
    assert sha(img) == golden["frames"][key]["sha"]


@pytest.mark.parametrize("order", [0, 1, 2])
def test_queue_orders_identical(gpu, mirt, golden, order):
    """MIRT_OPT_QUEUE_ORDER (the first bounces' queue order: auto, octant
    groups, tile order) changes only who walks which chain when: the golden
    1080p frame through the blocking call and through a device frame at the
    bench's 384-workgroup grid."""
    import torch
    abi = mirt.abi
    s, b = _scene(mirt, "render", 10000)
    gpu.upload(s, b)
    cam = mirt.default_camera()
    key = "1920x1080_render10000_d5_m1_b1_s1_c0_step1"
    out = torch.zeros((1080, 1920), dtype=torch.int32, device="cuda")
    try:
        gpu.set_option(abi.OPT_QUEUE_ORDER, order)
        assert gpu.get_option(abi.OPT_QUEUE_ORDER) == order
        img = gpu.render_frame(cam, 1920, 1080, depth=5, seed=1)
        gpu.set_option(abi.OPT_BOUNCE_BLOCKS, 384)
        gpu.render_frame_device(cam, mirt.frame_desc(1920, 1080, depth=5, seed=1), out.data_ptr(), None,
                                torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        with pytest.raises(mirt.MirtError):
            gpu.set_option(abi.OPT_QUEUE_ORDER, 3)
    finally:
        gpu.set_option(abi.OPT_QUEUE_ORDER, 0)
        gpu.set_option(abi.OPT_BOUNCE_BLOCKS, 0)
    assert sha(img) == golden["frames"][key]["sha"]
    dev = out.cpu().numpy().view(np.uint8).reshape(1080, 1920, 4)
    assert sha(dev) == golden["frames"][key]["sha"]


def test_traversal_v02_alias(gpu, mirt):
    """the mirt 0.2 header's MIRT_TRAV_WAVEFRONT (1) is accepted as
    a deprecated alias and reads back as 5; the retired ids stay errors."""
    abi = mirt.abi
    try:
        gpu.set_option(abi.OPT_TRAVERSAL, abi.TRAV_TILE)
        gpu.set_option(abi.OPT_TRAVERSAL, 1)
        assert gpu.get_option(abi.OPT_TRAVERSAL) == abi.TRAV_WAVEFRONT
        for bad in (2, 3, 4, 6):
            with pytest.raises(mirt.MirtError):
                gpu.set_option(abi.OPT_TRAVERSAL, bad)
    finally:
        gpu.set_option(abi.OPT_TRAVERSAL, abi.TRAV_WAVEFRONT)


def test_blocking_frame_into_registered_buffer(gpu, mirt, golden):
    """mirt_render_frame into the caller's own malloc'd buffer after
    mirt_host_register (main.c's frame buffer, page-locked in place) -- the
    kernels write the pixels straight into it (MIRT_OPT_ZERO_COPY) -- and
    into mirt_host_alloc memory: the golden frame; fresh and accumulating
    frames, depth 1 and 5, brute force, equal the copy path's and pageable
    memory's."""
    abi = mirt.abi
    s, b = _scene(mirt, "render", 10000)
    gpu.upload(s, b)
    cam = mirt.default_camera()
    page = np.zeros((1080, 1920, 4), np.uint8)
    hb = mirt.HostBuffer((1080, 1920, 4))
    mirt.host_register(page)
    try:
        assert gpu.get_option(abi.OPT_ZERO_COPY) == 1
        for dst in (page, hb.array):
            for _ in range(2):
                dst[:] = 0
                gpu.render_frame_into(cam, 1920, 1080, dst, depth=5, seed=1)
                assert sha(dst) == golden["frames"]["1920x1080_render10000_d5_m1_b1_s1_c0_step1"]["sha"]
        W, H = 640, 360
        small_page = np.zeros((H, W, 4), np.uint8)
        for kw in (dict(depth=5), dict(depth=1), dict(depth=5, use_bvh=False)):
            want = [gpu.render_frame(cam, W, H, seed=2, sample=k, accumulate=k > 0, frames=k + 1, **kw)
                    for k in range(3)]
            pinned = hb.array.reshape(-1)[:H * W * 4].reshape(H, W, 4)
            for zc in (1, 0):
                gpu.set_option(abi.OPT_ZERO_COPY, zc)
                for dst in (pinned, small_page):   # each a whole accumulation run from a fresh frame
                    for k in range(3):
                        gpu.render_frame_into(cam, W, H, dst, seed=2, sample=k, accumulate=k > 0, frames=k + 1, **kw)
                        assert (dst == want[k]).all(), (kw, zc, k)
    finally:
        gpu.set_option(abi.OPT_ZERO_COPY, 1)
        mirt.host_unregister(page)
        hb.close()


def test_cached_tree_renders_golden_frame(gpu, mirt, golden, tmp_path):
    """A scene uploaded from the tree cache file (mirt_bvh_build_flat_cached,
    second call = a load) renders the golden 1080p depth-5 frame."""
    path = tmp_path / "render10000.bvh"
    for want in (0, 1):
        s = mirt.create_random_spheres(10000, 1)
        b, cached = mirt.build_bvh_cached(path, s)
        assert cached == want
    gpu.upload(s, b)
    img = gpu.render_frame(mirt.default_camera(), 1920, 1080, depth=5, seed=1)
    assert sha(img) == golden["frames"]["1920x1080_render10000_d5_m1_b1_s1_c0_step1"]["sha"]


def test_per_ray_surface_matches_reference(mirt, small, golden):
    """include/mirt_dropin.h by value, one launch per call, against the
    reference's own outputs: get_camera_ray, ray_bvh_intersect on a pointer
    tree (object pointers into the caller's array), trace_ray (contract pixel
    = call order), ray_sphere_intersect and ray_aabb_intersect (empty boxes)."""
    import ctypes as C
    abi = mirt.abi
    L = mirt.load()
    assert L.mirt_dropin_init(0, 160, 90) == 0
    try:
        s = small["render_1000_1_pre"].copy()
        root = mirt.build_bvh_node(s)
        base = s.ctypes.data
        rays = small["hits_rays"]
        idx = list(range(0, 4000, 97)) + list(range(4000, len(rays)))[:60]
        want = small["hits_render_1000"]
        for i in idx:
            h = L.mirt_ray_bvh_intersect(abi.Ray.from_buffer_copy(rays[i].tobytes()), root)
            assert L.mirt_dropin_status() == 0
            assert h.hit_something == want[i]["hit"], i
            if h.hit_something:
                assert (h.object - base) // abi.SPHERE.itemsize == want[i]["sphere"], i
                assert np.float32(h.t).tobytes() == want[i]["t"].tobytes(), i
        L.mirt_dropin_rng(3, 0)
        tr = small["trace_d5_mode1"]
        for i in range(48):
            c = L.mirt_trace_ray(abi.Ray.from_buffer_copy(rays[i].tobytes()), C.c_void_p(base), len(s), 5, root)
            assert bytes(c) == tr[i].tobytes(), i
        ps, pw = small["pairs_spheres"], small["pairs_sphere_hits"]
        for i in range(0, 400, 7):
            sp = np.ascontiguousarray(ps[i:i + 1])
            h = L.mirt_ray_sphere_intersect(abi.Ray.from_buffer_copy(rays[i].tobytes()), C.c_void_p(sp.ctypes.data))
            assert h.hit_something == pw[i]["hit"] and (not h.hit_something or h.object == sp.ctypes.data), i
            if h.hit_something:
                assert np.float32(h.t).tobytes() == pw[i]["t"].tobytes(), i
        bx, bw = small["pairs_boxes"], small["pairs_box_hits"]
        for i in list(range(0, 70)) + list(range(70, 2000, 37)):
            a = L.mirt_ray_aabb_intersect(abi.Ray.from_buffer_copy(rays[i].tobytes()),
                                          abi.Aabb.from_buffer_copy(bx[i].tobytes()))
            assert a == bw[i], i
        cam = mirt.default_camera()
        cr = small["camrays_160x90_cam0"]       # rows 0, 1, 45, 89 of the reference's camera rays
        for ri, y in enumerate([0, 1, 45, 89]):
            for x in (0, 1, 79, 80, 159):
                u = np.float32((np.float32(x) / np.float32(160) - np.float32(0.5)) * (np.float32(160) / np.float32(90)))
                v = np.float32(np.float32(y) / np.float32(90) - np.float32(0.5))
                r = L.mirt_get_camera_ray(C.byref(cam), float(u), float(-v))
                assert bytes(r) == cr[ri, x].tobytes(), (y, x)
        mirt.free_bvh(root)
    finally:
        L.mirt_dropin_release()


def _bench_like_phantom_scene(mirt):
    """Three spheres at one centre (no SAH plane separates them: every
    candidate cost is NaN, bvh.c:139-141 falls back to x < 0.0 and all go
    left, so each level's right child is a 0-sphere leaf at &spheres[end])
    plus a fourth sphere OUTSIDE the build range, as benchmark.c:317 builds
    over [0, n - 1): the trailing 0-sphere leaves point at spheres[3], which
    hit.c:96-97 tests whenever the ray passes the cluster's box."""
    s = np.zeros(4, mirt.abi.SPHERE)
    for i in range(3):
        s[i]["center"] = (-1.0, 0.0, -10.0)
        s[i]["radius"] = 1.0
        s[i]["color"] = (200, 10 * i, 0, 255)
    s[3]["center"] = (5.0, 0.0, -10.0)
    s[3]["radius"] = 2.0
    s[3]["color"] = (0, 0, 250, 255)
    rays = np.zeros(6, mirt.abi.RAY)
    rays["origin"] = [(-10, 0.9, -10.9), (-10, -0.9, -9.1), (-10, 0.0, -10.0), (-10, 0.9, -9.1), (-10, 1.5, -10),
                      (-10, 0.95, -10.95)]
    rays["direction"] = (1.0, 0.0, 0.0)
    return s, rays


def test_orphan_phantom_leaf_is_tested(gpu, mirt, oracle):
    """A 0-sphere leaf pointing past its tree's range at a real sphere (the
    benchmark.c:317 build over [0, n - 1)) is tested as hit.c:96-97 does --
    the upload detects it and walks that tree in the reference's DFS order --
    for the batch call (array of n) and for the drop-in ray_bvh_intersect
    with the array declared (mirt_dropin_scene) or not (then spheres[n - 1]
    lies past what the tree spans: the never-hit sentinel, not read)."""
    import ctypes as C
    s, rays = _bench_like_phantom_scene(mirt)
    so = s.copy()
    t = oracle.build(so, 0, 3, 20)
    want4 = oracle.intersect(t, so, rays)
    want3 = oracle.intersect(t, so[:3], rays)
    oracle.free(t)
    assert (want4["sphere"] == 3).sum() >= 2 and not (want3["sphere"] == 3).any()   # the case is real
    root = mirt.build_bvh_node(s, 0, 3, 20)
    try:
        gpu.upload(s, root)
        assert gpu.closest_hit(rays).tobytes() == want4.tobytes()
        L = mirt.load()
        abi = mirt.abi
        base = s.ctypes.data
        for declared, want in ((False, want3), (True, want4)):
            assert L.mirt_dropin_scene(C.c_void_p(base) if declared else None, 4 if declared else 0) == 0
            L.mirt_dropin_invalidate()
            for i in range(len(rays)):
                h = L.mirt_ray_bvh_intersect(abi.Ray.from_buffer_copy(rays[i].tobytes()), root)
                assert L.mirt_dropin_status() == 0
                assert h.hit_something == want[i]["hit"], (declared, i)
                if h.hit_something:
                    assert (h.object - base) // abi.SPHERE.itemsize == want[i]["sphere"], (declared, i)
                    assert np.float32(h.t).tobytes() == want[i]["t"].tobytes(), (declared, i)
    finally:
        mirt.free_bvh(root)
        mirt.load().mirt_dropin_scene(None, 0)
        mirt.load().mirt_dropin_release()


def test_dropin_rebinds_after_free_and_rebuild(mirt, oracle):
    """benchmark.c:306-324's loop through the drop-in: free_bvh + free, then
    the next point's spheres and tree -- here in the SAME sphere buffer and
    with the same count, so the array pointer and count repeat and the root
    usually comes back at the old address; the drop-in's content
    fingerprint must re-upload (no mirt_dropin_invalidate), else it walks
    the freed tree. Every hit equals the oracle's on that point's scene."""
    import ctypes as C
    abi = mirt.abi
    L = mirt.load()
    buf = np.zeros(400, abi.SPHERE)
    base = buf.ctypes.data
    st = mirt.RandState(7)
    roots = []
    try:
        for n in (400, 400, 400, 300):
            s = mirt.create_benchmark_spheres(n, state=st)
            buf[:n] = s
            root = mirt.build_bvh_node(buf, 0, n - 1, 20)      # benchmark.c:317
            roots.append(root)
            rays = mirt.create_bench_rays(64, st)
            so = s.copy()
            t = oracle.build(so, 0, n - 1, 20)
            want = oracle.intersect(t, so, rays)
            oracle.free(t)
            for i in range(len(rays)):
                h = L.mirt_ray_bvh_intersect(abi.Ray.from_buffer_copy(rays[i].tobytes()), root)
                assert L.mirt_dropin_status() == 0
                assert h.hit_something == want[i]["hit"], (n, i)
                if h.hit_something:
                    assert (h.object - base) // abi.SPHERE.itemsize == want[i]["sphere"], (n, i)
                    assert np.float32(h.t).tobytes() == want[i]["t"].tobytes(), (n, i)
            mirt.free_bvh(root)                               # benchmark.c:323-324
            buf[:] = 0
        print("root addresses", [hex(r) for r in roots], "repeated:", len(set(roots)) < len(roots))
    finally:
        L.mirt_dropin_release()


def test_phantom_grazing_rays(gpu, mirt, oracle):
    """The fast walks drop 0-sphere leaves (render.hip dead_leaf): exact if a
    ray that hits a sphere always passes the box fl(c -+ r) of that sphere's
    own leaf under hit.c:49-82's division test. Rays aimed at the silhouettes
    (within 1e-3 .. 1e-6 of the radius) of the spheres that 0-sphere leaves of
    both kinds point at (mid == start: spheres[start]; mid == end: spheres[end],
    outside the leaf's subtree), from points inside the 0-sphere leaf's parent
    box: the ordered / pruned walks == the reference-order DFS walk == the
    oracle."""
    s, b = _scene(mirt, "render", 10000)
    nd = b.nodes
    empty = np.nonzero((nd["sphere"] >= 0) & ((nd["skip"] & mirt.abi.NODE_EMPTY) != 0))[0]
    assert len(empty) > 100
    # parent of every node: pre-order, inner i has children i + 1 and skip(i + 1)
    parent = np.full(len(nd), -1, np.int64)
    for i in np.nonzero(nd["sphere"] < 0)[0]:
        parent[i + 1] = i
        parent[nd["skip"][i + 1] & mirt.abi.SKIP_MASK] = i
    # the 0-sphere leaves that are their parent's right child point at
    # spheres[end] of the parent's range (mid == end)
    right = [e for e in empty if parent[e] >= 0 and e != parent[e] + 1]
    left = [e for e in empty if parent[e] >= 0 and e == parent[e] + 1]
    assert right and left
    rng = np.random.default_rng(11)
    pick = list(rng.choice(right, min(120, len(right)), replace=False)) + \
        list(rng.choice(left, min(120, len(left)), replace=False))
    rays = []
    for e in pick:
        j = nd["sphere"][e]
        if j >= len(s):
            continue
        p = nd[parent[e]]
        c = s[j]["center"].astype(np.float64)
        r = float(s[j]["radius"])
        for _ in range(8):
            o = rng.uniform(p["bmin"], p["bmax"])
            u = rng.normal(size=3)
            to = c - o
            to /= np.linalg.norm(to)
            u -= u.dot(to) * to
            u /= np.linalg.norm(u)
            tgt = c + u * r * (1.0 - 10.0 ** rng.uniform(-6, -3))
            d = tgt - o
            d /= np.linalg.norm(d)
            rays.append((o, d))
    ray = np.zeros(len(rays), mirt.abi.RAY)
    ray["origin"] = [o for o, _ in rays]
    ray["direction"] = [d for _, d in rays]
    gpu.upload(s, b)
    fast = gpu.closest_hit(ray)
    try:
        gpu.set_option(mirt.abi.OPT_ORDERED, 0)
        gpu.set_option(mirt.abi.OPT_PRUNE, 0)
        dfs = gpu.closest_hit(ray)
    finally:
        gpu.set_option(mirt.abi.OPT_ORDERED, 1)
        gpu.set_option(mirt.abi.OPT_PRUNE, 1)
    s2 = mirt.create_random_spheres(10000, 1)
    t = oracle.build(s2)
    want = oracle.intersect(t, s2, ray)
    oracle.free(t)
    assert dfs.tobytes() == want.tobytes()
    assert fast.tobytes() == want.tobytes()
    assert int(want["hit"].sum()) > len(ray) // 4


@pytest.mark.parametrize("batch,accumulate,direct", [(1, True, False), (4, True, False), (4, False, False),
                                                    (4, False, True), (3, True, True)])
def test_bench_launch_plan_displays(gpu, mirt, batch, accumulate, direct):
    """bench.py's timed loop through mirt_multi: `batch` successive frames per
    launch, launches rotating over four lanes (the lanes share one
    accumulation buffer, each context's bounce pass at the 1.5-per-CU grid
    mirt_multi sets for lanes > 1, the last launch on the full grid), every
    frame delivered to its own host buffer (gather or host-direct): each
    equals frame k of successive blocking calls on one ctx (accumulating:
    the display main.c:379-408 shows after frame k)."""
    s, b = _scene(mirt, "render", 10000)
    W, H, F = 320, 180, 12
    cam = mirt.default_camera()
    bufs = [mirt.HostBuffer((H, W, 4)) for _ in range(F)]
    try:
        with mirt.MultiRenderer([0], lanes=4, host_direct=direct) as m:
            m.upload(s, b)
            assert m.delivery == ("host-direct" if direct else "gather")
            # launches of `batch` frames; the display loop's first frame is a
            # fresh frame of its own (accumulate = 0 with several frames means
            # successive FRESH frames)
            starts = ([0] + list(range(1, F, batch))) if accumulate else list(range(0, F, batch))
            for i, f0 in enumerate(starts):
                k = (starts[i + 1] if i + 1 < len(starts) else F) - f0
                acc = accumulate and f0 > 0
                fd = mirt.frame_desc(W, H, depth=5, seed=1, sample=f0, accumulate=acc, frames=f0 + 1 if acc else 1)
                m.render_frames_async(cam, fd, bufs[f0:f0 + k], full_grid=f0 + k >= F)
            m.wait()
            got = [x.array.copy() for x in bufs]
    finally:
        for x in bufs:
            x.close()
    gpu.upload(s, b)
    for k in range(F):
        acc = accumulate and k > 0
        seq = gpu.render_frame(cam, W, H, depth=5, seed=1, sample=k, accumulate=acc, frames=k + 1 if acc else 1)
        assert (got[k] == seq).all(), k


@pytest.mark.parametrize("batch", [0, 1])
def test_leaf_batch_modes_identical(gpu, mirt, golden, small, batch):
    """The bounce walk with a step's leaf spheres loaded together
    (MIRT_OPT_LEAF_BATCH 1: bounce_kernel WALK 4, the default on trees past
    the L2) and without (0) renders every golden depth-5 BVH frame, including
    the 1M benchmark-sphere frame, byte for byte."""
    abi = mirt.abi
    cs = cams(mirt, small)
    try:
        n = 0
        for key in sorted(golden["frames"]):
            p = parse_frame_key(key)
            if p["depth"] < 2 or p["mode"] != 1 or not p["use_bvh"]:
                continue
            s, b = _scene(mirt, p["kind"], p["n"])
            gpu.upload(s, b)
            gpu.set_option(abi.OPT_LEAF_BATCH, batch)
            assert gpu.get_option(abi.OPT_LEAF_BATCH) == batch
            img = gpu.render_frame(cs[p["cam"]], p["W"], p["H"], depth=p["depth"], seed=p["seed"])[::p["step"]]
            assert sha(img) == golden["frames"][key]["sha"], key
            n += 1
        assert n >= 8
    finally:
        gpu.set_option(abi.OPT_LEAF_BATCH, 2)


@pytest.mark.parametrize("case", ["tiny_far", "huge", "offset"])
def test_bounded_slab_edge_scenes(gpu, mirt, oracle, case):
    """The bounce walks test the four-wide tree's boxes without margins: the
    boxes are grown by 2^-19 C at upload (C bounds every box and every sphere
    point) and a bounce ray whose origin lies beyond C takes the exact test.
    Scenes at the edges of that argument against the oracle, byte for byte:
    a tiny scene (C < 1, a growth of 2^-20) seen from 300x its size, benchmark
    spheres beyond the fp16 range (no growth: every bounce ray exact), and a
    cloud far from the origin (C set by the offset, not the spread).
    (Farther views of the tiny scene hit nothing in the reference either: its
    float discriminant loses the radius.)"""
    if case == "tiny_far":
        s = mirt.create_random_spheres(2000, 3)
        s["center"] *= np.float32(0.02)
        s["radius"] *= np.float32(0.02)
        cam = mirt.default_camera()
        cam.position = mirt.abi.Vec3(0.0, 0.1, 300.0)   # 300x the scene's scale (the growth is 2^-19 C)
        cam.fov = 0.3
    elif case == "huge":
        s = mirt.create_benchmark_spheres(3000, 5, world_size=2.0e5)
        s["radius"] = np.float32(4000.0)
        cam = mirt.default_camera()
        cam.position = mirt.abi.Vec3(0.0, 0.0, 3.0e5)
    else:
        s = mirt.create_random_spheres(2000, 4)
        s["center"][:, 0] += np.float32(3000.0)
        cam = mirt.default_camera()
        cam.position = mirt.abi.Vec3(3000.0, 4.0, 50.0)
    s2 = s.copy()
    gpu.upload(s, mirt.build_bvh(s))
    t = oracle.build(s2)
    try:
        for W, H, depth, seed in ((96, 54, 5, 1), (77, 45, 3, 2)):
            img = gpu.render_frame(cam, W, H, depth=depth, seed=seed)
            ref = oracle.render(cam, W, H, s2, t, depth=depth, use_bvh=True, mode=1, seed=seed)
            bad = int((img != ref).any(-1).sum())
            assert bad == 0, f"{case} {W}x{H} depth {depth}: {bad} pixels differ"
            assert len(np.unique(ref.reshape(-1, 4), axis=0)) > 50, case   # spheres in view, not just sky
    finally:
        oracle.free(t)
