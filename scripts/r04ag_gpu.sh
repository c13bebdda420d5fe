#!/bin/bash
# Round 4: the first bounces written with one atomic per workgroup in tile order (MIRT_PRIMARY_GROUP 2) against the octant grouping (1) and one atomic per wave (0):
# bounces costs and buys on the final kernels (MIRT_PRIMARY_GROUP 0 vs 1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04ag
mkdir -p $OUT
L="ab/libmirt_base.so ab/libmirt_pg0.so ab/libmirt_pg2.so"
timeout -k 10 500 python scripts/ab_libs.py $L --rounds 3 --steps 20 > $OUT/ab_10k.log 2>&1 || exit 1
grep -h '^{' $OUT/ab_10k.log | cut -c1-250
grep BEST $OUT/ab_*.log
timeout -k 10 500 python scripts/ab_libs.py $L --rounds 2 --steps 20 --workload 1080p_100k > $OUT/ab_100k.log 2>&1 || exit 1
grep BEST $OUT/ab_100k.log
