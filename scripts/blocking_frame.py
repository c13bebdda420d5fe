"""The reference's one-frame-at-a-time loop (main.c:350-421: render, then
SDL_RenderPresent) through the blocking call, by destination (VERDICT r3
"halve the blocking frame's overhead"):

  pageable      mirt_render_frame into a numpy array (the runtime stages the D2H)
  registered    the same numpy array after mirt_host_register (page-locked in
                place: the kernels write the pixels straight into it,
                MIRT_OPT_ZERO_COPY; registered_copy: one DMA after the kernels)
  pinned        mirt_render_frame into mirt_host_alloc memory (pinned_copy: DMA)
  kernels       the frame's kernels alone into device memory (one launch)

1080p / 10k depth 5 (bench.py's workload), median of 21 calls each, every
frame checked against the first. Prints one JSON line.
  python scripts/blocking_frame.py [--workload 1080p_10k]
"""
import argparse
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=21)
    a = ap.parse_args()
    import torch
    W, H = 1920, 1080
    s = m.create_random_spheres(10000, 1)
    b = m.build_bvh(s)
    r = m.Renderer(0)
    r.upload(s, b)
    cam = m.default_camera()

    def med(fn):
        fn()
        dts = []
        for _ in range(a.calls):
            t0 = time.perf_counter()
            fn()
            dts.append(time.perf_counter() - t0)
        return sorted(dts)[len(dts) // 2] * 1e3

    ref = r.render_frame(cam, W, H, depth=5, seed=1)
    out = {"workload": "1920x1080, 10000 spheres, depth 5 (blocking mirt_render_frame per frame)"}
    page = np.zeros((H, W, 4), np.uint8)
    ok = True
    out["pageable_ms"] = med(lambda: r.render_frame_into(cam, W, H, page, depth=5, seed=1))
    ok = ok and bool((page == ref).all())
    m.host_register(page)
    hb = m.HostBuffer((H, W, 4))
    try:
        for zc, sfx in ((1, ""), (0, "_copy")):
            r.set_option(m.abi.OPT_ZERO_COPY, zc)
            page[:] = 0
            out["registered" + sfx + "_ms"] = med(lambda: r.render_frame_into(cam, W, H, page, depth=5, seed=1))
            ok = ok and bool((page == ref).all())
            hb.array[:] = 0
            out["pinned" + sfx + "_ms"] = med(lambda: r.render_frame_into(cam, W, H, hb.array, depth=5, seed=1))
            ok = ok and bool((hb.array == ref).all())
    finally:
        r.set_option(m.abi.OPT_ZERO_COPY, 1)
        m.host_unregister(page)
        hb.close()
    d = torch.zeros((H, W), dtype=torch.int32, device="cuda")
    fd = m.frame_desc(W, H, depth=5, seed=1)
    st = torch.cuda.Stream()

    def kern():
        r.render_frame_device(cam, fd, d.data_ptr(), None, st.cuda_stream)
        st.synchronize()
    out["kernels_ms"] = med(kern)
    for k in ("pageable", "registered", "registered_copy", "pinned", "pinned_copy", "kernels"):
        out[k + "_mrays_s"] = round(W * H / out[k + "_ms"] / 1e3, 1)
        out[k + "_ms"] = round(out[k + "_ms"], 4)
    out["frames_equal"] = ok
    print(json.dumps(out), flush=True)
    r.close()


if __name__ == "__main__":
    main()
