#!/bin/bash
# Round 4: group drain for the last 2..4 rays of a bounce wave (out-of-line
# group_chain) against the solo drain alone; parity of the in-tree build
# (group drain on) first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=r04p
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
L="ab/libmirt_solo.so ab/libmirt_g2.so ab/libmirt_g4.so"
timeout -k 10 400 python scripts/ab_libs.py $L --rounds 3 --steps 20 > $OUT/ab_10k.log 2>&1 || exit 1
timeout -k 10 400 python scripts/ab_libs.py $L --rounds 2 --steps 20 --workload 1080p_100k > $OUT/ab_100k.log 2>&1 || exit 1
timeout -k 10 600 python scripts/ab_libs.py $L --rounds 1 --steps 20 --workload 4k_1m_4spp > $OUT/ab_4k1m.log 2>&1 || exit 1
grep BEST $OUT/ab_*.log
for lib in solo g4; do
  timeout -k 10 120 env MIRT_LIB=ab/libmirt_$lib.so python scripts/blocking_frame.py > $OUT/blocking_$lib.log 2>&1 || exit 1
  tail -1 $OUT/blocking_$lib.log | cut -c1-300
done
