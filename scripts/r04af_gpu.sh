#!/bin/bash
# Round 4: what the camera-packet kernel's octant grouping of the first
# bounces costs and buys on the final kernels (MIRT_PRIMARY_GROUP 0 vs 1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04af
mkdir -p $OUT
L="ab/libmirt_base.so ab/libmirt_pg0.so"
timeout -k 10 500 python scripts/ab_libs.py $L --rounds 3 --steps 20 > $OUT/ab_10k.log 2>&1 || exit 1
grep -h '^{' $OUT/ab_10k.log | cut -c1-250
grep BEST $OUT/ab_*.log
