#!/bin/bash
# Round 5, session bl: two camera packets per wave (MIRT_PACKET_HALVES: the
# wave's lower and upper 32 lanes walk separately, both halves' PNodes
# requested under one scalar wait) at 8 and 7 waves per SIMD against the base
# build: parity suites on each variant, then the A/B at 1080p/10k, 1080p/100k
# and 4K/1M (the serial primary launch and the pipelined frame loop).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05bl
mkdir -p $OUT
for v in hv8 hv7; do
  MIRT_LIB=$PWD/ab/libmirt_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_full_frames.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_$v.log 2>&1 || { echo "parity $v failed"; tail -30 $OUT/pytest_$v.log; exit 1; }
  tail -1 $OUT/pytest_$v.log
done
for wl in 1080p_10k 1080p_100k 4k_1m_4spp; do
  timeout -k 10 600 python scripts/ab_libs.py ab/libmirt_base.so ab/libmirt_hv8.so ab/libmirt_hv7.so --workload $wl --steps 20 --rounds 2 > $OUT/ab_$wl.log 2>&1 || { echo "ab $wl failed"; tail -20 $OUT/ab_$wl.log; exit 1; }
  grep BEST $OUT/ab_$wl.log
done
