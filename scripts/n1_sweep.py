"""The N = 1 frame loop through mirt_multi under a grid of settings, each in
a FRESH process (GPU_MAX_HW_QUEUES is read when the HIP runtime starts):
lanes, hardware queues, delivery (host memory / device only), steps.

    python scripts/n1_sweep.py --lanes 4,8 --queues 4,16 --steps 20,100
"""
import argparse
import itertools
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import importlib.util, json, os, sys
spec = importlib.util.spec_from_file_location("bench", os.path.join(sys.argv[1], "bench.py"))
bench = importlib.util.module_from_spec(spec); spec.loader.exec_module(bench)
lanes, steps, dev_only, batch = int(sys.argv[2]), int(sys.argv[3]), sys.argv[4] == "1", int(sys.argv[5])
spheres, bvh, _ = bench.make_scene()
cam = bench.mirt.default_camera()
m = bench.open_multi(1, lanes, False, spheres, bvh, 384 if lanes > 1 else 0, [])
bufs = bench.host_bufs(lanes, batch)
t = bench.timed_loop(m, cam, bench.plan(0, 5, batch), bench.plan(5, steps, batch), bufs, 5, device_only=dev_only)
t2 = bench.timed_loop(m, cam, bench.plan(0, 5, batch), bench.plan(5, steps, batch), bufs, 5, device_only=dev_only)
print(json.dumps({"mrays_s": [round(1920 * 1080 * steps / x / 1e6, 1) for x in (t, t2)]}))
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lanes", default="4")
    ap.add_argument("--queues", default="4,16")
    ap.add_argument("--steps", default="20")
    ap.add_argument("--batch", default="1")
    ap.add_argument("--device-only", default="0,1")
    a = ap.parse_args()
    for lanes, q, steps, dev, batch in itertools.product(a.lanes.split(","), a.queues.split(","), a.steps.split(","),
                                                         a.device_only.split(","), a.batch.split(",")):
        env = dict(os.environ, GPU_MAX_HW_QUEUES=q)
        p = subprocess.run([sys.executable, "-c", CHILD, ROOT, lanes, steps, dev, batch], capture_output=True,
                           text=True, env=env, timeout=300)
        line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
        res = json.loads(line[-1]) if p.returncode == 0 and line else {"error": p.stderr[-400:]}
        print(json.dumps({"lanes": int(lanes), "hw_queues": int(q), "steps": int(steps), "batch": int(batch),
                          "delivery": "device-only" if dev == "1" else "host", **res}), flush=True)


if __name__ == "__main__":
    main()
