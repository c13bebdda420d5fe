"""Host cost of issuing one launch through mirt_multi from one thread, by
rank count: n ranks on the ONE GPU of this box (same-device ranks, the
host-direct delivery: every rank's render + its strided copies), `lanes`
launches enqueued back to back with no lane to wait for (each lane used once
per burst), 4 frames per launch as bench.py's N >= 4 schedule. At N GPUs the
host issues this for every launch, so per frame it must stay well under the
N-GPU frame period (~0.13 ms at N = 8, 1080p/10k).

    python scripts/host_issue.py [--ranks 1,2,4,8]
"""
import argparse
import importlib.util
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
bench = importlib.util.module_from_spec(spec)
spec.loader.exec_module(bench)
mirt = bench.mirt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", default="1,2,4,8")
    ap.add_argument("--lanes", type=int, default=8)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--bursts", type=int, default=5)
    ap.add_argument("--opt", action="append", default=[])
    a = ap.parse_args()
    W, H = 1920, 1080
    s = mirt.create_random_spheres(10000, 1)
    b = mirt.build_bvh(s)
    cam = mirt.default_camera()
    for n in (int(x) for x in a.ranks.split(",")):
        m = mirt.MultiRenderer([0] * n, lanes=a.lanes, host_direct=True)
        m.upload(s, b)
        for ov in a.opt:
            o, v = (int(t) for t in ov.split("="))
            m.set_option(o, v)
        bufs = bench.host_bufs(a.lanes, a.batch) if False else [[mirt.HostBuffer((H, W, 4)) for _ in range(a.batch)]
                                                                for _ in range(a.lanes)]
        per = []
        for burst in range(a.bursts + 1):
            m.wait()
            for lane in range(a.lanes):
                fd = mirt.frame_desc(W, H, depth=5, seed=1, sample=(burst * a.lanes + lane) * a.batch)
                t0 = time.perf_counter()
                m.render_frames_async(cam, fd, bufs[m.launches % a.lanes], nframes=a.batch)
                if burst:
                    per.append(time.perf_counter() - t0)
        m.wait()
        m.close()
        for lane in bufs:
            for x in lane:
                x.close()
        med = statistics.median(per) * 1e3
        print(json.dumps({"ranks": n, "lanes": a.lanes, "frames_per_launch": a.batch, "options": a.opt,
                          "enqueue_ms_per_launch_median": round(med, 4),
                          "enqueue_ms_per_launch_p90": round(sorted(per)[int(0.9 * len(per))] * 1e3, 4),
                          "host_ms_per_frame": round(med / a.batch, 4)}), flush=True)


if __name__ == "__main__":
    main()
