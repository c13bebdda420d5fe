"""The host-direct delivery's copy shape, issued the way mirt_multi issues it
(hipMemcpy2DAsync from the compact slab into the interleaved host frame,
page-locked by mirt_host_alloc), against a contiguous copy of the same bytes,
the same rows split over 2 / 4 streams, and one hipMemcpyAsync per row block:
is the strided DMA limited per row or per byte?

    python scripts/d2h2d_probe.py [--world 8]
"""
import argparse
import ctypes
import importlib
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
mirt = importlib.import_module("cs201_sah-bvh_ray_tracer_amd")
W, H, RB = 1920, 1080, 8
D2H = 2   # hipMemcpyDeviceToHost


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--reps", type=int, default=200)
    a = ap.parse_args()
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy2DAsync.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
                                     ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    world = a.world
    blocks = (H // RB) // world                      # full blocks of shard 0
    row_bytes = RB * W * 4
    slab = torch.zeros((blocks * RB, W), dtype=torch.int32, device="cuda")
    frame = mirt.HostBuffer((H, W, 4))
    contig = mirt.HostBuffer((blocks * RB, W, 4))
    streams = [torch.cuda.Stream() for _ in range(4)]
    dst, src = frame.array.ctypes.data, slab.data_ptr()
    nbytes = blocks * row_bytes

    def timeit(fn):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / a.reps

    def d2d_2d(k):
        def fn():
            per = (blocks + k - 1) // k
            for i in range(k):
                b0, nb = i * per, min(per, blocks - i * per)
                if nb <= 0:
                    continue
                rc = hip.hipMemcpy2DAsync(dst + b0 * world * row_bytes, world * row_bytes, src + b0 * row_bytes,
                                          row_bytes, row_bytes, nb, D2H, streams[i].cuda_stream)
                assert rc == 0, rc
        return fn

    def per_block():
        for b in range(blocks):
            rc = hip.hipMemcpyAsync(dst + b * world * row_bytes, src + b * row_bytes, row_bytes, D2H,
                                    streams[0].cuda_stream)
            assert rc == 0, rc

    def contiguous():
        rc = hip.hipMemcpyAsync(contig.array.ctypes.data, src, nbytes, D2H, streams[0].cuda_stream)
        assert rc == 0, rc

    out = {"world": world, "rows": blocks, "row_bytes": row_bytes, "bytes": nbytes}
    for name, fn in (("contiguous", contiguous), ("strided_2d_1stream", d2d_2d(1)), ("strided_2d_2streams", d2d_2d(2)),
                     ("strided_2d_4streams", d2d_2d(4)), ("per_block_1stream", per_block)):
        t = timeit(fn)
        out[name] = {"ms": round(t * 1e3, 4), "gbs": round(nbytes / t / 1e9, 2)}
    print(json.dumps(out), flush=True)
    frame.close()
    contig.close()


if __name__ == "__main__":
    main()
