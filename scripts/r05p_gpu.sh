#!/bin/bash
# Round 5, session p: camera-packet prefetch through the vector path
# (MIRT_PACKET_PREFETCH) at 7 and 8 waves per SIMD against the base build:
# parity suites on each variant, then the A/B at 1080p/10k and 4K/1M.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05p
mkdir -p $OUT
for v in pf7 pf8; do
  MIRT_LIB=$PWD/ab/libmirt_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_full_frames.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_$v.log 2>&1 || { echo "parity $v failed"; tail -30 $OUT/pytest_$v.log; exit 1; }
  tail -1 $OUT/pytest_$v.log
done
for wl in 1080p_10k 4k_1m_4spp; do
  timeout -k 10 500 python scripts/ab_libs.py ab/libmirt_base.so ab/libmirt_pf7.so ab/libmirt_pf8.so --workload $wl --steps 20 --rounds 2 > $OUT/ab_$wl.log 2>&1 || { echo "ab $wl failed"; tail -20 $OUT/ab_$wl.log; exit 1; }
  grep BEST $OUT/ab_$wl.log
done
