"""Does hipPointerGetAttributes (mirt_multi's page-locked check of every
output, render.hip host_mapped) wait for the device? Times the query while a
frame stalled 300 ms (MIRT_OPT_DEBUG_STALL_MS) is in flight, and in a quiet
process, on page-locked and pageable memory."""
import ctypes
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
m = importlib.import_module("cs201_sah-bvh_ray_tracer_amd")


def main():
    hip = ctypes.CDLL("libamdhip64.so")
    attr = ctypes.create_string_buffer(512)

    def query(p):
        t0 = time.perf_counter()
        rc = hip.hipPointerGetAttributes(attr, ctypes.c_void_p(p))
        dt = time.perf_counter() - t0
        hip.hipGetLastError()
        return rc, dt * 1e6

    hb = m.HostBuffer((1080, 1920, 4))
    page = np.zeros((1080, 1920, 4), np.uint8)
    s = m.create_random_spheres(1000, 1)
    b = m.build_bvh(s)
    r = m.Renderer(0)
    r.upload(s, b)
    quiet = {"pinned_us": [round(query(hb.array.ctypes.data)[1], 1) for _ in range(5)],
             "pageable_us": [round(query(page.ctypes.data)[1], 1) for _ in range(5)]}
    r.set_option(m.abi.OPT_DEBUG_STALL_MS, 300)
    fd = m.frame_desc(160, 90, depth=5)
    out = m.HostBuffer((90, 160, 4))
    t0 = time.perf_counter()
    r.render_frame_async(m.default_camera(), fd, out)
    enq = time.perf_counter() - t0
    busy = {"pinned_us": [round(query(hb.array.ctypes.data)[1], 1) for _ in range(5)],
            "pageable_us": [round(query(page.ctypes.data)[1], 1) for _ in range(5)]}
    t1 = time.perf_counter()
    r.wait()
    print(json.dumps({"quiet": quiet, "while_frame_in_flight": busy, "enqueue_ms": round(enq * 1e3, 3),
                      "wait_after_queries_ms": round((time.perf_counter() - t1) * 1e3, 1)}), flush=True)
    r.set_option(m.abi.OPT_DEBUG_STALL_MS, 0)
    out.close()
    hb.close()
    r.close()


if __name__ == "__main__":
    main()
