"""A/B of libmirt builds (kernel variants of the same ABI): for each library,
the golden 1080p depth-5 frame must match, then bench.py's device numbers.

    python scripts/ab_libs.py ab/libmirt_base.so ab/libmirt_x.so [--workload 1080p_10k] [--rounds 2]
    python scripts/ab_libs.py ab/libmirt_x.so ab/libmirt_x.so@21=1 ...   (LIB@OPT=VAL[,OPT=VAL]: bench.py --opt)

Each library runs in its own process (MIRT_LIB), rounds interleaved.
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHECK = r'''
import hashlib, importlib, json, sys, torch
sys.path.insert(0, %r)
m = importlib.import_module("cs201_sah-bvh_ray_tracer_amd")
g = json.load(open(%r))
s = m.create_random_spheres(10000, 1); b = m.build_bvh(s)
r = m.Renderer(0); r.upload(s, b)
img = r.render_frame(m.default_camera(), 1920, 1080, depth=5, seed=1)
ok = hashlib.sha256(img.tobytes()).hexdigest() == g["frames"]["1920x1080_render10000_d5_m1_b1_s1_c0_step1"]["sha"]
print("golden", ok); sys.exit(0 if ok else 3)
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--workload", default="1080p_10k")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--steps", type=int, default=100)
    a = ap.parse_args()
    res = {lib: [] for lib in a.libs}
    for spec in dict.fromkeys(x.split("@")[0] for x in a.libs):
        lib = spec
        env = dict(os.environ, MIRT_LIB=os.path.abspath(lib))
        p = subprocess.run([sys.executable, "-c", CHECK % (ROOT, os.path.join(ROOT, "tests/golden/golden.json"))],
                           env=env, capture_output=True, text=True, timeout=300)
        print(lib, p.stdout.strip(), p.stderr.strip()[-300:], flush=True)
        if p.returncode:
            sys.exit(p.returncode)
    for _ in range(a.rounds):
        for lib in a.libs:
            path, _, opts = lib.partition("@")
            env = dict(os.environ, MIRT_LIB=os.path.abspath(path))
            extra = [x for o in opts.split(",") if o for x in ("--opt", o)]
            p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu", "--no-host",
                                "--workload", a.workload, "--steps", str(a.steps)] + extra, env=env,
                               capture_output=True, text=True, timeout=600)
            if p.returncode:
                print(lib, "bench failed", p.stderr[-1000:])
                sys.exit(p.returncode)
            d = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
            # round 4: the timed launches' HIP-event times live under reference_work
            rl = d.get("reference_work") or d["roofline"]
            sl = rl.get("serial_launch", rl)      # bench.py before round 3 kept these at the top level
            b_ms = rl.get("bounce_launch_ms_under_overlap", rl.get("kernel_ms"))
            p_ms = rl.get("primary_launch_ms_under_overlap", rl.get("primary_kernel_ms"))
            res[lib].append((d["value"], b_ms, p_ms, sl["frame_ms"], d["depth1_mrays_s"]))
            print(json.dumps({"lib": lib, "value": d["value"], "device_resident": d.get("device_resident_mrays_s"),
                              "bounce_ms": b_ms,
                              "primary_ms": p_ms, "frame_ms": sl["frame_ms"],
                              "serial_bounce_ms": sl.get("bounce_ms"), "serial_primary_ms": sl.get("primary_ms"),
                              "depth1": d["depth1_mrays_s"]}), flush=True)
    for lib, v in res.items():
        if not v:
            continue
        best = max(v)
        print("BEST", lib, "value %.1f bounce %.4f primary %.4f serial frame %.4f depth1 %.1f" % best)


if __name__ == "__main__":
    main()
