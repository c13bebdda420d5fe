#!/bin/bash
# Round 4: alternating queue control blocks zeroed by the previous frame's
# camera-packet pass (MIRT_QCTL_PARITY 1) instead of a memset dispatch per
# frame (0) -- the GPU suite through the variant, then the A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04aq
mkdir -p $OUT
timeout -k 10 600 env MIRT_LIB=ab/libmirt_qp1.so python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
L="ab/libmirt_qp0.so ab/libmirt_qp1.so"
timeout -k 10 500 python scripts/ab_libs.py $L --rounds 3 --steps 20 > $OUT/ab_10k.log 2>&1 || exit 1
timeout -k 10 500 python scripts/ab_libs.py $L --rounds 2 --steps 20 --workload 1080p_100k > $OUT/ab_100k.log 2>&1 || exit 1
grep BEST $OUT/ab_*.log
for lib in qp0 qp1; do
  timeout -k 10 120 env MIRT_LIB=ab/libmirt_$lib.so python scripts/blocking_frame.py > $OUT/blocking_$lib.log 2>&1 || exit 1
  echo "$lib $(tail -1 $OUT/blocking_$lib.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["pinned_ms"], d["pageable_ms"], d["kernels_ms"], d["frames_equal"])')"
done
