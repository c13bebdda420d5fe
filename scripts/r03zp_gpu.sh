#!/bin/bash
# Packed brute-force loop shared with the frame path (BVH off): the GPU
# suite on the in-tree library, then a 1080p / 10k brute-force depth-5 frame
# timed for the scalar and the packed builds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r03zp
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -n 15 "$OUT/pytest_gpu.log"; exit 1; }
tail -n 1 "$OUT/pytest_gpu.log"
for lib in base bpk base bpk; do
  MIRT_LIB=ab/libmirt_$lib.so timeout -k 10 300 python - >> "$OUT/brute_frame.log" 2>&1 <<PY || exit 1
import importlib, sys, time, torch
sys.path.insert(0, ".")
m = importlib.import_module("cs201_sah-bvh_ray_tracer_amd")
s = m.create_random_spheres(10000, 1); b = m.build_bvh(s)
r = m.Renderer(0); r.upload(s, b)
cam = m.default_camera()
r.render_frame(cam, 1920, 1080, depth=5, seed=1, use_bvh=False)
t0 = time.perf_counter(); n = 3
for _ in range(n): r.render_frame(cam, 1920, 1080, depth=5, seed=1, use_bvh=False)
dt = (time.perf_counter() - t0) / n
print("$lib", "brute-force 1080p/10k depth-5 frame", round(dt * 1e3, 2), "ms", round(1920 * 1080 / dt / 1e6, 1), "Mrays/s", flush=True)
PY
done
cat "$OUT/brute_frame.log" | grep brute
