#!/bin/bash
# Round 5, session q: pricing a three-load node format by
# its inverse -- one MORE load instruction per four-wide visit (x1: a word of
# the same node; x2: a word of the neighbouring HNode) against the base build,
# at 1080p/10k and 4K/1M 4 spp.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05q
mkdir -p $OUT
for wl in 4k_1m_4spp 1080p_10k; do
  timeout -k 10 540 python scripts/ab_libs.py ab/libmirt_base.so ab/libmirt_x1.so ab/libmirt_x2.so --workload $wl --steps 20 --rounds 2 > $OUT/ab_$wl.log 2>&1 || { echo "ab $wl failed"; tail -20 $OUT/ab_$wl.log; exit 1; }
  grep BEST $OUT/ab_$wl.log
done
