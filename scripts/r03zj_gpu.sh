#!/bin/bash
# Packed-fp32 brute-force loop: benchmark-mode parity tests on the in-tree
# library, then the published sweep (1K-10M, device times) for the scalar and
# the packed builds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r03zj
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_bench_mode.py tests/test_gpu_parity.py -m gpu -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -n 5 "$OUT/pytest.log"; exit 1; }
tail -n 1 "$OUT/pytest.log"
for lib in base packed; do
  MIRT_LIB=ab/libmirt_$lib.so timeout -k 10 300 python -u scripts/bench_mode_published.py --counts 1000,10000,100000,1000000,10000000 --check-rays 64 --out "$OUT/bm_$lib" > "$OUT/bm_$lib.log" 2>&1 || { tail -n 5 "$OUT/bm_$lib.log"; exit 1; }
  grep -o '"spheres": [0-9]*\|"time_no_bvh_s": [0-9.e-]*\|"any_hit_equals_oracle": [a-z]*' "$OUT/bm_$lib.log" | paste - - - 
done
