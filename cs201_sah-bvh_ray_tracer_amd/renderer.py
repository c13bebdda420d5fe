"""Python host side of the render path, mirroring the reference's interface.

Reference call surface -> here (all compute goes through libmirt.so):

  srand / rand (glibc, main.c:90)             RandState
  create_random_sphere x N (sphere.c:52-59,   create_random_spheres(n, seed)
    main.c:218-221)
  create_benchmark_sphere (sphere.c:34-41,    create_benchmark_spheres(n, seed)
    benchmark.c:307-314)
  camera init (main.c:203-211) / camera_update default_camera() / camera_update(cam)
    (camera.c:10-18)
  build_bvh_node (bvh.c:117-209)               build_bvh(spheres, start, end, depth) -> Bvh
                                               build_bvh_cached(path, spheres, ...) (tree cache file)
                                               build_bvh_node(...) -> pointer tree (drop-in)
  get_camera_ray (ray.c:17-32) per pixel       Renderer.get_camera_rays(cam, W, H)
  trace_ray (renderer.c:21-77) per ray         Renderer.trace_ray(rays, depth, ...)
  pixel loop main.c:356-374 / 379-408          Renderer.render_frame(cam, W, H, ...)
  ray_bvh_intersect (hit.c:91-109)             Renderer.ray_bvh_intersect(rays)
  ray_sphere_intersect (hit.c:19-39)           Renderer.ray_sphere_intersect(rays, spheres)
  ray_aabb_intersect (hit.c:49-82)             Renderer.ray_aabb_intersect(rays, boxes)

Errors raise MirtError (the reference only printf's); there is no CPU path.
"""
import ctypes as C
import os

import numpy as np

from . import abi
from .lib import MirtError, check, load

ptr = abi.ptr


class RandState:
    """glibc srand()/rand() (TYPE_3), restated in libmirt."""

    def __init__(self, seed=1):
        self.st = abi.RandState()
        load().mirt_srand(C.byref(self.st), seed)

    def rand(self):
        return load().mirt_rand(C.byref(self.st))


def create_random_spheres(n, seed=1, state=None):
    """srand(seed) then n x create_random_sphere() (main.c:218-221)."""
    st = state or RandState(seed)
    out = np.zeros(n, abi.SPHERE)
    check(load().mirt_scene_random(C.byref(st.st), ptr(out), n), "mirt_scene_random")
    return out


def create_benchmark_spheres(n, seed=1, world_size=1000.0, state=None):
    """srand(seed) then the benchmark.c:307-314 sphere loop."""
    st = state or RandState(seed)
    out = np.zeros(n, abi.SPHERE)
    check(load().mirt_scene_benchmark(C.byref(st.st), ptr(out), n, world_size), "mirt_scene_benchmark")
    return out


def create_bench_rays(n, state):
    """n rays of benchmark.c:176-185 (origin 0, normalised random direction)
    drawn from `state` (a RandState continuing the scene's glibc stream)."""
    out = np.zeros(n, abi.RAY)
    check(load().mirt_bench_rays(C.byref(state.st), ptr(out), n), "mirt_bench_rays")
    return out


def default_camera():
    cam = abi.Camera()
    load().mirt_camera_default(C.byref(cam))
    return cam


def camera_update(cam):
    load().mirt_camera_update(C.byref(cam))
    return cam


class Bvh:
    """A flattened tree (abi.NODE array) plus the leaf sphere counts it came from."""

    def __init__(self, nodes):
        self.nodes = nodes

    def __len__(self):
        return len(self.nodes)


def build_bvh(spheres, start=0, end=None, depth=0):
    """build_bvh_node (bvh.c:117) straight into the flat layout; reorders
    `spheres` in place exactly like the reference."""
    assert spheres.dtype == abi.SPHERE and spheres.flags["C_CONTIGUOUS"]
    end = len(spheres) if end is None else end
    out = C.c_void_p()
    cnt = C.c_int()
    L = load()
    check(L.mirt_bvh_build_flat(ptr(spheres), start, end, depth, C.byref(out), C.byref(cnt)), "mirt_bvh_build_flat")
    try:
        buf = (C.c_char * (cnt.value * abi.NODE.itemsize)).from_address(out.value)
        nodes = np.frombuffer(bytes(buf), dtype=abi.NODE).copy()
    finally:
        L.mirt_bvh_free_flat(out)
    return Bvh(nodes)


def validate_bvh(nodes, num_spheres):
    """mirt_bvh_validate_flat: raises MirtError unless `nodes` (abi.NODE) is a
    well-formed flat pre-order tree over num_spheres spheres."""
    nodes = np.ascontiguousarray(nodes, dtype=abi.NODE)
    check(load().mirt_bvh_validate_flat(ptr(nodes) if len(nodes) else None, len(nodes), num_spheres),
          "mirt_bvh_validate_flat")


def build_bvh_cached(path, spheres, start=0, end=None, depth=0):
    """build_bvh through a flattened-tree cache file (mirt_bvh_build_flat_cached):
    returns (Bvh, cached) with cached 1 = loaded from `path`, 0 = built and
    written, -1 = built, file not written. `spheres` ends up reordered exactly
    as build_bvh leaves it either way."""
    assert spheres.dtype == abi.SPHERE and spheres.flags["C_CONTIGUOUS"]
    end = len(spheres) if end is None else end
    out = C.c_void_p()
    cnt = C.c_int()
    cached = C.c_int()
    L = load()
    check(L.mirt_bvh_build_flat_cached(os.fsencode(path), ptr(spheres), start, end, depth, C.byref(out),
                                       C.byref(cnt), C.byref(cached)), "mirt_bvh_build_flat_cached")
    try:
        buf = (C.c_char * (cnt.value * abi.NODE.itemsize)).from_address(out.value)
        nodes = np.frombuffer(bytes(buf), dtype=abi.NODE).copy()
    finally:
        L.mirt_bvh_free_flat(out)
    return Bvh(nodes), cached.value


def build_bvh_node(spheres, start=0, end=None, depth=0):
    """Drop-in build_bvh_node: returns the reference-layout pointer tree
    (free with free_bvh)."""
    end = len(spheres) if end is None else end
    root = load().mirt_build_bvh_node(ptr(spheres), start, end, depth)
    if not root:
        raise MirtError(load().mirt_last_error().decode())
    return root


def free_bvh(root):
    load().mirt_free_bvh(root)


def flatten_bvh(root, spheres):
    """Flatten a pointer tree (ours or the reference's) into a Bvh."""
    L = load()
    n = L.mirt_bvh_count(root)
    nodes = np.zeros(n, abi.NODE)
    check(L.mirt_bvh_flatten(root, ptr(spheres), ptr(nodes), n), "mirt_bvh_flatten")
    return Bvh(nodes)


def frame_desc(width, height, depth=5, use_bvh=True, seed=1, sample=0, accumulate=False, frames=1,
               row_block=8, shard=0, num_shards=1, samples=1, jitter=False, lead_skip=0):
    fd = abi.FrameDesc()
    fd.width, fd.height, fd.max_depth, fd.use_bvh = width, height, depth, int(use_bvh)
    fd.seed, fd.sample, fd.accumulate, fd.frames = seed, sample, int(accumulate), frames
    fd.row_block, fd.shard, fd.num_shards = row_block, shard, num_shards
    fd.samples = samples
    fd.jitter = int(jitter)
    fd.lead_skip = lead_skip
    return fd


def shard_rows(fd):
    """Image rows a shard renders, in its compacted order."""
    L = load()
    n = check(L.mirt_shard_rows(C.byref(fd), None), "mirt_shard_rows")
    rows = np.zeros(n, np.int32)
    L.mirt_shard_rows(C.byref(fd), ptr(rows))
    return rows


def host_register(arr):
    """Page-lock a C-contiguous numpy array in place (mirt_host_register):
    blocking frames copied into it become one DMA. host_unregister before the
    array is released."""
    assert arr.flags["C_CONTIGUOUS"]
    check(load().mirt_host_register(ptr(arr), arr.nbytes), "mirt_host_register")


def host_unregister(arr):
    check(load().mirt_host_unregister(ptr(arr)), "mirt_host_unregister")


class HostBuffer:
    """Page-locked host memory (mirt_host_alloc) viewed as a numpy array."""

    def __init__(self, shape, dtype=np.uint8):
        self.L = load()
        nbytes = int(np.prod(shape)) * np.dtype(dtype).itemsize
        p = C.c_void_p()
        check(self.L.mirt_host_alloc(nbytes, C.byref(p)), "mirt_host_alloc")
        self.p = p
        buf = (C.c_char * max(nbytes, 1)).from_address(p.value)
        self.array = np.frombuffer(buf, dtype=dtype, count=int(np.prod(shape))).reshape(shape)

    def close(self):
        if self.p:
            self.array = None
            self.L.mirt_host_free(self.p)
            self.p = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Renderer:
    """One device context (mirt_ctx) with a resident scene."""

    def __init__(self, device=0):
        self.L = load()
        h = C.c_void_p()
        check(self.L.mirt_create(device, C.byref(h)), "mirt_create")
        self.h = h
        self.device = device
        self.num_spheres = -1

    def close(self):
        if self.h:
            self.L.mirt_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ---- scene
    def upload(self, spheres, bvh=None):
        """Upload the (post-build) spheres and a Bvh, a pointer tree, or None."""
        spheres = np.ascontiguousarray(spheres, abi.SPHERE)
        if bvh is None:
            check(self.L.mirt_scene_upload_flat(self.h, ptr(spheres), len(spheres), None, 0), "upload")
        elif isinstance(bvh, Bvh):
            check(self.L.mirt_scene_upload_flat(self.h, ptr(spheres), len(spheres), ptr(bvh.nodes), len(bvh.nodes)),
                  "mirt_scene_upload_flat")
        else:
            check(self.L.mirt_scene_upload(self.h, ptr(spheres), len(spheres), bvh), "mirt_scene_upload")
        self.num_spheres = len(spheres)

    # ---- frames
    def render_frame(self, cam, width, height, depth=5, use_bvh=True, seed=1, sample=0, accumulate=False,
                     frames=1, row_block=8, shard=0, num_shards=1, samples=1, jitter=False):
        """main.c:356-374 (fresh) or main.c:379-408 (accumulate) for one shard;
        returns (rows, width, 4) uint8 in the shard's row order. samples > 1:
        that many successive frames (RNG samples sample, sample + 1, ...) in
        one launch, accumulated; returns the display after the last."""
        fd = frame_desc(width, height, depth, use_bvh, seed, sample, accumulate, frames, row_block, shard,
                        num_shards, samples, jitter)
        n = check(self.L.mirt_shard_rows(C.byref(fd), None), "mirt_shard_rows")
        out = np.zeros((n, width, 4), np.uint8)
        check(self.L.mirt_render_frame(self.h, C.byref(cam), C.byref(fd), ptr(out)), "mirt_render_frame")
        return out

    def render_frame_into(self, cam, width, height, out, depth=5, use_bvh=True, seed=1, sample=0, accumulate=False,
                          frames=1, samples=1, jitter=False):
        """render_frame into a caller-given C-contiguous uint8 array (pageable,
        registered or page-locked) of height x width x 4."""
        fd = frame_desc(width, height, depth, use_bvh, seed, sample, accumulate, frames, 8, 0, 1, samples, jitter)
        assert out.flags["C_CONTIGUOUS"] and out.nbytes >= width * height * 4
        check(self.L.mirt_render_frame(self.h, C.byref(cam), C.byref(fd), ptr(out)), "mirt_render_frame")
        return out

    def render_frame_async(self, cam, fd, out):
        """Enqueue the frame and its D2H copy into `out` (a HostBuffer, or any
        C-contiguous uint8 array of the shard's rows x width x 4) on the ctx's
        own stream; `out` is complete after wait()."""
        arr = out.array if isinstance(out, HostBuffer) else out
        n = check(self.L.mirt_shard_rows(C.byref(fd), None), "mirt_shard_rows")
        if arr.nbytes < n * fd.width * 4 or not arr.flags["C_CONTIGUOUS"]:
            raise MirtError(f"render_frame_async: output holds {arr.nbytes} bytes, the shard needs {n * fd.width * 4}")
        check(self.L.mirt_render_frame_async(self.h, C.byref(cam), C.byref(fd), ptr(arr)), "mirt_render_frame_async")

    def wait(self):
        """Block until the ctx's stream is idle (mirt_ctx_wait)."""
        check(self.L.mirt_ctx_wait(self.h), "mirt_ctx_wait")

    def render_frame_device(self, cam, fd, d_out, d_acc=None, stream=None):
        """Enqueue a frame into device memory (integer device pointers)."""
        check(self.L.mirt_render_frame_device(self.h, C.byref(cam), C.byref(fd), C.c_void_p(d_out),
                                              C.c_void_p(d_acc) if d_acc else None,
                                              C.c_void_p(stream or 0)), "mirt_render_frame_device")

    def share_accum(self, owner):
        """Use `owner`'s accumulation buffer (mirt_ctx_share_accum): the ctxs
        of one accumulating display loop with frames in flight; None: a
        private buffer again."""
        check(self.L.mirt_ctx_share_accum(self.h, owner.h if owner is not None else None), "mirt_ctx_share_accum")

    def accum(self, count):
        out = np.zeros(count, np.float32)
        check(self.L.mirt_accum_download(self.h, ptr(out), count), "mirt_accum_download")
        return out

    def count_frame(self, cam, width, height, depth=5, use_bvh=True, seed=1, sample=0, row_block=8, shard=0,
                    num_shards=1, samples=1, jitter=False):
        """Work of one launch (samples frames): rays, node tests, sphere tests, hits."""
        fd = frame_desc(width, height, depth, use_bvh, seed, sample, False, 1, row_block, shard, num_shards,
                        samples, jitter)
        c = abi.Counts()
        check(self.L.mirt_count_frame(self.h, C.byref(cam), C.byref(fd), C.byref(c)), "mirt_count_frame")
        return {k: getattr(c, k) for k, _ in abi.Counts._fields_}

    def set_option(self, option, value):
        """abi.OPT_TRAVERSAL (abi.TRAV_*) / abi.OPT_FAST_SLAB (0/1): speed only."""
        check(self.L.mirt_set_option(self.h, option, value), "mirt_set_option")

    def get_option(self, option):
        return check(self.L.mirt_get_option(self.h, option), "mirt_get_option")

    def bounce_stats(self, cam, width, height, depth=5, seed=1, sample=0, shard=0, num_shards=1):
        """Per-wave diagnostic of the bounce kernel: uint64 array of (iterations,
        walking lanes summed, iterations after the queue ran dry, their lanes,
        t_start, t_dry, t_end [10 ns ticks], longest chain << 32 | longest walk,
        quad-drain iterations, t_quad_start, DFS-segment fallback lane-steps,
        fallbacks entered)."""
        fd = frame_desc(width, height, depth, True, seed, sample, False, 1, 8, shard, num_shards)
        n = -self.L.mirt_bounce_stats(self.h, C.byref(cam), C.byref(fd), None, 0)
        if n <= 0:
            check(-n, "mirt_bounce_stats")
        out = np.zeros((n, 12), np.uint64)
        check(self.L.mirt_bounce_stats(self.h, C.byref(cam), C.byref(fd), ptr(out), n), "mirt_bounce_stats")
        return out

    def wave_stats(self, cam, width, height, depth=5, use_bvh=True, seed=1, sample=0, row_block=8, shard=0,
                   num_shards=1):
        """Per-wave (8x8 tile) diagnostic: array of (tile, steps, start, end),
        start/end in 10 ns ticks of the device's constant clock."""
        fd = frame_desc(width, height, depth, use_bvh, seed, sample, False, 1, row_block, shard, num_shards)
        n = -self.L.mirt_wave_stats(self.h, C.byref(cam), C.byref(fd), None, 0)
        out = np.zeros((n, 4), np.uint32)
        check(self.L.mirt_wave_stats(self.h, C.byref(cam), C.byref(fd), ptr(out), n), "mirt_wave_stats")
        return out

    @property
    def stream_handle(self):
        """The ctx's own hipStream_t (int)."""
        return self.L.mirt_ctx_stream(self.h) or 0

    @property
    def last_kernel_ms(self):
        return self.L.mirt_last_kernel_ms(self.h)

    def last_phase_ms(self):
        """(primary ms, bounce ms) of the last wavefront-schedule frame; waits for it."""
        out = (C.c_float * 2)()
        check(self.L.mirt_last_phase_ms(self.h, out), "mirt_last_phase_ms")
        return float(out[0]), float(out[1])

    def phase_log(self, n=64):
        """(primary ms, bounce ms) of each of the ctx's last <= n wavefront
        frames, oldest first, from HIP events on each frame's own stream
        (durations under whatever overlap the frames ran with); waits."""
        out = (C.c_float * (2 * n))()
        k = check(self.L.mirt_phase_log(self.h, out, n), "mirt_phase_log")
        return [(float(out[2 * j]), float(out[2 * j + 1])) for j in range(k)]

    def bvh_overlay(self, cam, width, height, max_levels=-1):
        """The BVH debug view (bvh_visualiser.c:16-126) of the uploaded tree:
        (height, width, 4) uint8."""
        out = np.zeros((height, width, 4), np.uint8)
        check(self.L.mirt_bvh_overlay(self.h, C.byref(cam), width, height, max_levels, ptr(out)), "mirt_bvh_overlay")
        return out

    # ---- per-ray surface (batched)
    def get_camera_rays(self, cam, width, height, row_block=8, shard=0, num_shards=1):
        fd = frame_desc(width, height, 1, True, 1, 0, False, 1, row_block, shard, num_shards)
        n = check(self.L.mirt_shard_rows(C.byref(fd), None), "mirt_shard_rows")
        out = np.zeros((n, width), abi.RAY)
        check(self.L.mirt_camera_rays(self.h, C.byref(cam), C.byref(fd), ptr(out)), "mirt_camera_rays")
        return out

    def trace_ray(self, rays, depth=5, use_bvh=True, seed=1, sample=0):
        rays = np.ascontiguousarray(rays, abi.RAY)
        out = np.zeros((len(rays), 4), np.uint8)
        check(self.L.mirt_trace_rays(self.h, ptr(rays), len(rays), depth, int(use_bvh), seed, sample, ptr(out)),
              "mirt_trace_rays")
        return out

    def closest_hit(self, rays, use_bvh=True):
        rays = np.ascontiguousarray(rays, abi.RAY)
        out = np.zeros(len(rays), abi.HIT)
        check(self.L.mirt_intersect_rays(self.h, ptr(rays), len(rays), int(use_bvh), ptr(out)),
              "mirt_intersect_rays")
        return out

    def any_hit(self, rays, use_bvh=False):
        """int32 per ray: 1 if it hits some sphere (benchmark.c:190-199
        brute force; with use_bvh, ray_bvh_intersect's hit_something)."""
        rays = np.ascontiguousarray(rays, abi.RAY)
        out = np.zeros(len(rays), np.int32)
        check(self.L.mirt_any_hit_rays(self.h, ptr(rays), len(rays), int(use_bvh), ptr(out)), "mirt_any_hit_rays")
        return out

    def ray_bvh_intersect(self, rays):
        return self.closest_hit(rays, True)

    def ray_sphere_intersect(self, rays, spheres):
        rays = np.ascontiguousarray(rays, abi.RAY)
        spheres = np.ascontiguousarray(spheres, abi.SPHERE)
        out = np.zeros(len(rays), abi.HIT)
        check(self.L.mirt_sphere_pairs(self.h, ptr(rays), ptr(spheres), len(rays), ptr(out)), "mirt_sphere_pairs")
        return out

    def ray_aabb_intersect(self, rays, boxes):
        rays = np.ascontiguousarray(rays, abi.RAY)
        boxes = np.ascontiguousarray(boxes, abi.AABB)
        out = np.zeros(len(rays), np.int32)
        check(self.L.mirt_aabb_pairs(self.h, ptr(rays), ptr(boxes), len(rays), ptr(out)), "mirt_aabb_pairs")
        return out


class MultiRenderer:
    """One frame loop over several GPUs from this process (include/mirt_multi.h,
    SURVEY §8(b) mirt_init(num_gpus)): interleaved row blocks per rank, the
    slabs gathered to rank 0 over RCCL (distinct devices) or by device copies
    ("copy": forced, or a device listed twice -- n shards on one GPU), or with
    host_direct every rank's blocks copied straight into the host frame;
    `lanes` launches in flight, each of one or more frames. Frames equal
    Renderer.render_frame's on one GPU."""

    def __init__(self, devices, lanes=1, copy=False, host_direct=False, queue_ahead=False):
        self.L = load()
        devs = (C.c_int * len(devices))(*devices)
        h = C.c_void_p()
        flags = ((abi.MULTI_COPY if copy else 0) | (abi.MULTI_HOST_DIRECT if host_direct else 0)
                 | (abi.MULTI_QUEUE_AHEAD if queue_ahead else 0))
        check(self.L.mirt_multi_create(devs, len(devices), lanes, flags, C.byref(h)), "mirt_multi_create")
        self.h = h
        self.devices = list(devices)
        self.lanes = self.L.mirt_multi_lanes(h)   # launch slots (2 x lanes with queue_ahead)
        self.launches = 0   # launch k runs on lane k % lanes (mirt_multi's rotation)

    def close(self):
        if self.h:
            self.L.mirt_multi_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def backend(self):
        return self.L.mirt_multi_backend(self.h).decode()

    @property
    def delivery(self):
        return self.L.mirt_multi_delivery(self.h).decode()

    @property
    def size(self):
        return self.L.mirt_multi_size(self.h)

    @property
    def failed(self):
        return self.L.mirt_multi_failed(self.h) == 1

    def ctx(self, lane, rank):
        """(lane, rank)'s mirt_ctx handle (owned by the multi renderer)."""
        return self.L.mirt_multi_ctx(self.h, lane, rank)

    def phase_log(self, lane, rank, n):
        """mirt_phase_log of (lane, rank)'s context: [primary_ms, bounce_ms] of its last n frames."""
        buf = (C.c_float * (2 * n))()
        got = check(self.L.mirt_phase_log(self.ctx(lane, rank), buf, n), "mirt_phase_log")
        return [(buf[2 * i], buf[2 * i + 1]) for i in range(got)]

    def upload(self, spheres, bvh):
        spheres = np.ascontiguousarray(spheres, abi.SPHERE)
        if isinstance(bvh, Bvh):
            check(self.L.mirt_multi_scene_upload_flat(self.h, ptr(spheres), len(spheres), ptr(bvh.nodes),
                                                      len(bvh.nodes)), "mirt_multi_scene_upload_flat")
        else:
            check(self.L.mirt_multi_scene_upload(self.h, ptr(spheres), len(spheres), bvh), "mirt_multi_scene_upload")

    def set_option(self, option, value):
        """MULTI_OPT_* (timeout, emulation) or a MIRT_OPT_* for every context."""
        check(self.L.mirt_multi_set_option(self.h, option, value), "mirt_multi_set_option")

    def get_option(self, option):
        return check(self.L.mirt_multi_get_option(self.h, option), "mirt_multi_get_option")

    def emulate(self, world, rank):
        """Measurement only (one rank): play shard `rank` of a frame split
        `world` ways (MIRT_MULTI_OPT_EMULATE_*); frames are then incomplete."""
        self.set_option(abi.MULTI_OPT_EMULATE_WORLD, world)
        self.set_option(abi.MULTI_OPT_EMULATE_RANK, rank)

    def render_frame(self, cam, width, height, depth=5, use_bvh=True, seed=1, sample=0, accumulate=False, frames=1,
                     row_block=8, samples=1, jitter=False):
        """The whole frame (height, width, 4) uint8, blocking."""
        fd = frame_desc(width, height, depth, use_bvh, seed, sample, accumulate, frames, row_block, 0, 1, samples,
                        jitter)
        out = np.zeros((height, width, 4), np.uint8)
        check(self.L.mirt_multi_render_frame(self.h, C.byref(cam), C.byref(fd), ptr(out)), "mirt_multi_render_frame")
        self.launches += 1
        return out

    @staticmethod
    def _host(out, fd):
        arr = out.array if isinstance(out, HostBuffer) else out
        if arr.nbytes < fd.width * fd.height * 4 or not arr.flags["C_CONTIGUOUS"]:
            raise MirtError("mirt_multi: output too small or not contiguous")
        return arr

    def render_frame_async(self, cam, fd, out):
        """Enqueue a whole frame into `out` (HostBuffer or uint8 array of
        height x width x 4) on the next lane; complete after wait()."""
        arr = self._host(out, fd)
        check(self.L.mirt_multi_render_frame_async(self.h, C.byref(cam), C.byref(fd), ptr(arr)),
              "mirt_multi_render_frame_async")
        self.launches += 1

    def render_frames_async(self, cam, fd, outs, nframes=None, full_grid=False):
        """One launch of len(outs) successive frames (RNG samples fd.sample + j)
        on the next lane, frame j into outs[j]; outs None: `nframes` frames
        left on the devices. Complete after wait() (or the lane's next launch)."""
        n = len(outs) if outs is not None else int(nframes or 1)
        if outs is not None:
            arrs = [self._host(o, fd) for o in outs]
            cp = (C.c_void_p * n)(*[a.ctypes.data for a in arrs])
        else:
            cp = None
        check(self.L.mirt_multi_render_frames_async(self.h, C.byref(cam), C.byref(fd), n,
                                                    abi.MULTI_FULL_GRID if full_grid else 0, cp),
              "mirt_multi_render_frames_async")
        self.launches += 1

    def wait(self):
        check(self.L.mirt_multi_wait(self.h), "mirt_multi_wait")

    def stats(self):
        """mirt_multi_get_stats as a dict (RCCL calls issued, copies, launches)."""
        st = abi.MultiStats()
        check(self.L.mirt_multi_get_stats(self.h, C.byref(st)), "mirt_multi_get_stats")
        return {k: int(getattr(st, k)) for k, _ in abi.MultiStats._fields_}

    def read_gathered(self, shard, rows, width, frame=0, lane=-1):
        """Test hook: shard `shard`'s compact rows (rows x width RGBA8) of
        frame `frame` as they arrived in device 0's gather buffer in the last
        launch (lane -1) or lane `lane`'s."""
        out = np.zeros((rows, width, 4), np.uint8)
        check(self.L.mirt_multi_read_gathered(self.h, lane, shard, frame, ptr(out), out.nbytes),
              "mirt_multi_read_gathered")
        return out
