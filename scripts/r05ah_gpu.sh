#!/bin/bash
# Round 5, session ah: non-temporal moves of the bounce queue's records
# (MIRT_QUEUE_NT) against the base build at 1080p/10k, 1080p/100k, 4K/1M.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05ah
mkdir -p $OUT
timeout -k 10 400 python scripts/ab_libs.py ab/libmirt_base.so ab/libmirt_nt.so --workload 1080p_10k --steps 20 --rounds 3 > $OUT/ab_10k.log 2>&1 || { echo "ab 10k failed"; tail -5 $OUT/ab_10k.log; exit 1; }
grep BEST $OUT/ab_10k.log
for wl in 1080p_100k 4k_1m_4spp; do
  timeout -k 10 500 python scripts/ab_libs.py ab/libmirt_base.so ab/libmirt_nt.so --workload $wl --steps 20 --rounds 2 > $OUT/ab_$wl.log 2>&1 || { echo "ab $wl failed"; tail -5 $OUT/ab_$wl.log; exit 1; }
  grep BEST $OUT/ab_$wl.log
done
