"""numpy/ctypes mirror of include/mirt.h (the C-ABI of the render path).

Every dtype here is byte-compatible with the struct of the same name in
include/mirt.h, which in turn is layout-compatible with the reference's own
types (vec3.h:3-7, sphere.h:7-11, ray.h:5-8, camera.h:5-14, bvh.h:7-18,
hit.h:8-14).
"""
import ctypes as C

import numpy as np

VEC3 = ("<f4", (3,))

SPHERE = np.dtype([("center", *VEC3), ("radius", "<f4"), ("color", "u1", (4,))])   # 20 B
RAY = np.dtype([("origin", *VEC3), ("direction", *VEC3)])                           # 24 B
AABB = np.dtype([("min", *VEC3), ("max", *VEC3)])                                    # 24 B
HIT = np.dtype([("t", "<f4"), ("point", *VEC3), ("normal", *VEC3),
                ("hit", "<i4"), ("sphere", "<i4"), ("pad", "<i4")])                   # 40 B
NODE = np.dtype([("bmin", *VEC3), ("bmax", *VEC3), ("sphere", "<i4"), ("skip", "<u4")])  # 32 B
CAMERA = np.dtype([("position", *VEC3), ("forward", *VEC3), ("right", *VEC3), ("up", *VEC3),
                   ("yaw", "<f4"), ("pitch", "<f4"), ("fov", "<f4"), ("move", "<i4")])   # 64 B

NODE_EMPTY = 0x80000000
SKIP_MASK = 0x7FFFFFFF

assert SPHERE.itemsize == 20 and RAY.itemsize == 24 and AABB.itemsize == 24
assert HIT.itemsize == 40 and NODE.itemsize == 32 and CAMERA.itemsize == 64


class Vec3(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float)]


class Camera(C.Structure):
    """camera.h:5-14"""
    _fields_ = [("position", Vec3), ("forward", Vec3), ("right", Vec3), ("up", Vec3),
                ("yaw", C.c_float), ("pitch", C.c_float), ("fov", C.c_float), ("move", C.c_int)]

    def to_numpy(self):
        return np.frombuffer(bytes(self), dtype=CAMERA)[0]

    @classmethod
    def from_numpy(cls, rec):
        return cls.from_buffer_copy(np.asarray(rec, dtype=CAMERA).tobytes())


class Ray(C.Structure):
    """ray.h:5-8 (by value in the per-ray drop-in calls)"""
    _fields_ = [("origin", Vec3), ("direction", Vec3)]


class Aabb(C.Structure):
    """bvh.h:7-10"""
    _fields_ = [("min", Vec3), ("max", Vec3)]


class Rgba8(C.Structure):
    """SDL_Color"""
    _fields_ = [("r", C.c_uint8), ("g", C.c_uint8), ("b", C.c_uint8), ("a", C.c_uint8)]


class HitRecord(C.Structure):
    """hit.h:8-14 (object: pointer into the caller's sphere array)"""
    _fields_ = [("t", C.c_float), ("point", Vec3), ("normal", Vec3), ("hit_something", C.c_int),
                ("object", C.c_void_p)]


class RandState(C.Structure):
    """glibc TYPE_3 rand() state (mirt_rand_state)."""
    _fields_ = [("r", C.c_int32 * 34), ("f", C.c_int32), ("b", C.c_int32)]


class FrameDesc(C.Structure):
    """mirt_frame_desc"""
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("max_depth", C.c_int32),
                ("use_bvh", C.c_int32), ("seed", C.c_uint64), ("sample", C.c_uint32),
                ("accumulate", C.c_int32), ("frames", C.c_int32), ("row_block", C.c_int32),
                ("shard", C.c_int32), ("num_shards", C.c_int32), ("samples", C.c_int32),
                ("jitter", C.c_int32), ("lead_skip", C.c_int32)]


class Counts(C.Structure):
    """mirt_counts"""
    _fields_ = [("rays", C.c_uint64), ("nodes", C.c_uint64), ("spheres", C.c_uint64), ("hits", C.c_uint64),
                ("lane_steps", C.c_uint64), ("nodes_primary", C.c_uint64), ("spheres_primary", C.c_uint64),
                ("hits_primary", C.c_uint64)]


class MultiStats(C.Structure):
    """mirt_multi_stats (include/mirt_multi.h)"""
    _fields_ = [("launches", C.c_uint64), ("comm_inits", C.c_uint64), ("rccl_groups", C.c_uint64),
                ("rccl_sends", C.c_uint64), ("rccl_recvs", C.c_uint64), ("rccl_bytes", C.c_uint64),
                ("device_copies", C.c_uint64)]


def default_camera():
    """main.c:203-211: position (0,4,50), looking down -z, fov 45, yaw -pi."""
    cam = Camera()
    cam.position = Vec3(0.0, 4.0, 50.0)
    cam.forward = Vec3(0.0, 0.0, -1.0)
    cam.right = Vec3(1.0, 0.0, 0.0)
    cam.up = Vec3(0.0, 1.0, 0.0)
    cam.yaw = np.float32(-np.pi)
    cam.pitch = 0.0
    cam.fov = 45.0
    cam.move = 0
    return cam


def ptr(a):
    """ctypes void* of a contiguous numpy array (None passes through)."""
    if a is None:
        return None
    assert a.flags["C_CONTIGUOUS"]
    return C.c_void_p(a.ctypes.data)


# (name, restype, argtypes) of every symbol include/mirt.h declares.
P = C.c_void_p
I = C.c_int
SIGNATURES = [
    ("mirt_version", C.c_char_p, []),
    ("mirt_last_error", C.c_char_p, []),
    ("mirt_srand", None, [P, C.c_uint]),
    ("mirt_rand", I, [P]),
    ("mirt_scene_random", I, [P, P, I]),
    ("mirt_scene_benchmark", I, [P, P, I, C.c_float]),
    ("mirt_bench_rays", I, [P, P, I]),
    ("mirt_camera_default", None, [P]),
    ("mirt_camera_update", None, [P]),
    ("mirt_build_bvh_node", P, [P, I, I, I]),
    ("mirt_free_bvh", None, [P]),
    ("mirt_bvh_count", I, [P]),
    ("mirt_bvh_flatten", I, [P, P, P, I]),
    ("mirt_bvh_build_flat", I, [P, I, I, I, C.POINTER(P), C.POINTER(I)]),
    ("mirt_bvh_free_flat", None, [P]),
    ("mirt_bvh_validate_flat", I, [P, I, I]),
    ("mirt_bvh_build_flat_cached", I, [C.c_char_p, P, I, I, I, C.POINTER(P), C.POINTER(I), C.POINTER(I)]),
    ("mirt_create", I, [I, C.POINTER(P)]),
    ("mirt_destroy", None, [P]),
    ("mirt_scene_upload", I, [P, P, I, P]),
    ("mirt_scene_upload_flat", I, [P, P, I, P, I]),
    ("mirt_shard_rows", I, [P, P]),
    ("mirt_render_frame", I, [P, P, P, P]),
    ("mirt_render_frame_device", I, [P, P, P, P, P, P]),
    ("mirt_render_frame_async", I, [P, P, P, P]),
    ("mirt_ctx_wait", I, [P]),
    ("mirt_host_alloc", I, [C.c_size_t, C.POINTER(P)]),
    ("mirt_host_free", None, [P]),
    ("mirt_host_register", I, [P, C.c_size_t]),
    ("mirt_host_unregister", I, [P]),
    ("mirt_accum_download", I, [P, P, C.c_size_t]),
    ("mirt_ctx_share_accum", I, [P, P]),
    ("mirt_trace_rays", I, [P, P, I, I, I, C.c_uint64, C.c_uint32, P]),
    ("mirt_trace_rays_at", I, [P, P, I, I, I, C.c_uint64, C.c_uint32, C.c_uint32, P]),
    ("mirt_camera_rays_uv", I, [P, P, I, I, P, I, P]),
    ("mirt_bvh_overlay", I, [P, P, I, I, I, P]),
    ("mirt_intersect_rays", I, [P, P, I, I, P]),
    ("mirt_any_hit_rays", I, [P, P, I, I, P]),
    ("mirt_sphere_pairs", I, [P, P, P, I, P]),
    ("mirt_aabb_pairs", I, [P, P, P, I, P]),
    ("mirt_camera_rays", I, [P, P, P, P]),
    ("mirt_count_frame", I, [P, P, P, P]),
    ("mirt_wave_stats", I, [P, P, P, P, I]),
    ("mirt_ctx_stream", P, [P]),
    ("mirt_last_kernel_ms", C.c_float, [P]),
    ("mirt_last_phase_ms", I, [P, C.POINTER(C.c_float)]),
    ("mirt_phase_log", I, [P, C.POINTER(C.c_float), I]),
    ("mirt_bounce_stats", I, [P, P, P, P, I]),
    ("mirt_set_option", I, [P, I, I]),
    ("mirt_get_option", I, [P, I]),
    # include/mirt_dropin.h: the per-ray surface
    ("mirt_dropin_init", I, [I, I, I]),
    ("mirt_dropin_release", None, []),
    ("mirt_dropin_rng", None, [C.c_uint64, C.c_uint32]),
    ("mirt_dropin_scene", I, [P, I]),
    ("mirt_dropin_invalidate", None, []),
    ("mirt_dropin_status", I, []),
    ("mirt_get_camera_ray", Ray, [P, C.c_float, C.c_float]),
    ("mirt_trace_ray", Rgba8, [Ray, P, I, I, P]),
    ("mirt_ray_sphere_intersect", HitRecord, [Ray, P]),
    ("mirt_ray_aabb_intersect", I, [Ray, Aabb]),
    ("mirt_ray_bvh_intersect", HitRecord, [Ray, P]),
    # include/mirt_multi.h: one frame loop over several GPUs (RCCL gather)
    ("mirt_multi_create", I, [P, I, I, I, C.POINTER(P)]),
    ("mirt_multi_destroy", None, [P]),
    ("mirt_multi_size", I, [P]),
    ("mirt_multi_lanes", I, [P]),
    ("mirt_multi_backend", C.c_char_p, [P]),
    ("mirt_multi_delivery", C.c_char_p, [P]),
    ("mirt_multi_failed", I, [P]),
    ("mirt_multi_ctx", P, [P, I, I]),
    ("mirt_multi_set_option", I, [P, I, I]),
    ("mirt_multi_get_option", I, [P, I]),
    ("mirt_multi_scene_upload", I, [P, P, I, P]),
    ("mirt_multi_scene_upload_flat", I, [P, P, I, P, I]),
    ("mirt_multi_render_frame", I, [P, P, P, P]),
    ("mirt_multi_render_frame_async", I, [P, P, P, P]),
    ("mirt_multi_render_frames_async", I, [P, P, P, I, I, C.POINTER(P)]),
    ("mirt_multi_wait", I, [P]),
    ("mirt_multi_get_stats", I, [P, P]),
    ("mirt_multi_read_gathered", I, [P, I, I, I, P, C.c_size_t]),
]

OPT_TRAVERSAL, OPT_FAST_SLAB, OPT_BLOCK_WAVES, OPT_DEFER, OPT_BOUNCE_THRESHOLD, OPT_PRUNE, OPT_ORDERED = (
    1, 2, 3, 4, 5, 6, 7)
OPT_BOUNCE_BLOCKS, OPT_QUAD_DRAIN, OPT_LEAF_BATCH, OPT_QUAD_BATCH, OPT_ZERO_COPY = 9, 11, 14, 15, 17
OPT_QUEUE_ORDER, OPT_DEBUG_STALL_MS = 18, 19
TRAV_TILE, TRAV_WAVEFRONT = 0, 5
MULTI_COPY, MULTI_HOST_DIRECT, MULTI_QUEUE_AHEAD = 1, 2, 4
MULTI_FULL_GRID = 1
MULTI_OPT_TIMEOUT_MS, MULTI_OPT_EMULATE_WORLD, MULTI_OPT_EMULATE_RANK, MULTI_OPT_DIRECT_COPY = 256, 257, 258, 259
MULTI_OPT_COPY_STREAM = 260
MULTI_OPT_GATHER_SELF, MULTI_OPT_LEAD_SKIP = 261, 262
