#!/bin/bash
# Round 4: bounce-pass pixel stores queued per wave in LDS (one store
# instruction per 64 pixels) -- parity of the in-tree build, then the blocking
# frame (zero-copy into host memory) and the pipelined bench A/B against the
# committed solo-drain build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=r04u
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for lib in solo pq; do
  timeout -k 10 120 env MIRT_LIB=ab/libmirt_$lib.so python scripts/blocking_frame.py > $OUT/blocking_$lib.log 2>&1 || exit 1
  tail -1 $OUT/blocking_$lib.log | cut -c1-400
done
L="ab/libmirt_solo.so ab/libmirt_pq.so ab/libmirt_nopq.so"
timeout -k 10 400 python scripts/ab_libs.py $L --rounds 3 --steps 20 > $OUT/ab_10k.log 2>&1 || exit 1
timeout -k 10 400 python scripts/ab_libs.py $L --rounds 2 --steps 20 --workload 1080p_100k > $OUT/ab_100k.log 2>&1 || exit 1
grep BEST $OUT/ab_*.log
