"""The N = 1 frame loop of bench.py through mirt_multi with or without
MIRT_MULTI_QUEUE_AHEAD, for a HIP API trace (which host call blocks):

    rocprofv3 --hip-trace --stats -d gpurun_out/x -- python scripts/qa_probe.py 1 [COPY_STREAM]
"""
import importlib.util
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
bench = importlib.util.module_from_spec(spec)
spec.loader.exec_module(bench)


def main():
    ahead = len(sys.argv) > 1 and sys.argv[1] == "1"
    cs = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    spheres, bvh, _ = bench.make_scene()
    cam = bench.mirt.default_camera()
    m = bench.open_multi(1, 4, False, spheres, bvh, 384, [], ahead=ahead)
    m.set_option(bench.mirt.abi.MULTI_OPT_COPY_STREAM, cs)
    bufs = bench.host_bufs(m.lanes, 1)
    bench.prime(m, cam, bufs, 1)
    for _ in range(2):
        el = bench.timed_loop(m, cam, bench.plan(0, 5, 1), bench.plan(5, 20, 1), bufs, 5)
        enq = sorted(bench.ENQUEUE)
        print(json.dumps({"ahead": ahead, "copy_stream": cs, "mrays_s": round(1920 * 1080 * 20 / el / 1e6, 1),
                          "enqueue_ms": [round(x * 1e3, 3) for x in bench.ENQUEUE]}), flush=True)
    m.close()
    bench.close_bufs(bufs)


if __name__ == "__main__":
    t0 = time.time()
    main()
