"""MI355X-native primary-ray render path of the CS201 SAH-BVH sphere ray tracer.

Import with importlib (the directory name is not an identifier):

    mirt = importlib.import_module("cs201_sah-bvh_ray_tracer_amd")

Layout:
  csrc/        HIP kernels (render.hip, trace.h) and host C++ (BVH build,
               scene inputs) compiled into libmirt.so, the C ABI of
               include/mirt.h
  abi.py       numpy/ctypes mirror of include/mirt.h
  lib.py       loader (no fallback: missing library -> MirtError)
  renderer.py  the reference's call surface (trace_ray, build_bvh_node, ...)
  shard.py     row-block sharding of a frame over ranks + RCCL gather
  benchmark.py the reference's benchmark mode (benchmark.c) as batched launches
"""
from . import abi
from .lib import LIB_PATH, MirtError, build, load
from .renderer import (Bvh, HostBuffer, MultiRenderer, host_register, host_unregister, RandState, Renderer, build_bvh, build_bvh_cached, build_bvh_node, camera_update,
                       create_bench_rays, create_benchmark_spheres, create_random_spheres, default_camera,
                       flatten_bvh,
                       frame_desc, free_bvh, shard_rows, validate_bvh)

__all__ = ["abi", "LIB_PATH", "MirtError", "build", "load", "Bvh", "HostBuffer", "MultiRenderer", "host_register", "host_unregister", "RandState", "Renderer", "build_bvh", "build_bvh_cached",
           "build_bvh_node", "camera_update", "create_bench_rays", "create_benchmark_spheres", "create_random_spheres",
           "default_camera", "flatten_bvh", "frame_desc", "free_bvh", "shard_rows", "validate_bvh"]
