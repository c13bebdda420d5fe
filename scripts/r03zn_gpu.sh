#!/bin/bash
# Quad-per-ray BVH batches: the GPU suite on the in-tree library, then the
# published benchmark-mode sweep (1K-10M) for one ray per lane / per quad.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r03zn
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -n 15 "$OUT/pytest_gpu.log"; exit 1; }
tail -n 1 "$OUT/pytest_gpu.log"
for lib in base quad; do
  MIRT_LIB=ab/libmirt_$lib.so timeout -k 10 300 python -u scripts/bench_mode_published.py --counts 1000,10000,100000,1000000,10000000 --check-rays 256 --out "$OUT/bm_$lib" > "$OUT/bm_$lib.log" 2>&1 || { tail -n 5 "$OUT/bm_$lib.log"; exit 1; }
  grep -o '"spheres": [0-9]*\|"time_bvh_s": [0-9.e-]*\|"bvh_hits_equal_oracle": [a-z]*' "$OUT/bm_$lib.log" | paste - - -
done
