#!/bin/bash
# Round 5, session j: where the continuation queue's time goes (variants).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05j
mkdir -p "$OUT"
for v in cq_lane cqv1 cqv2 cqv3; do
  MIRT_LIB=$PWD/ab/libmirt_$v.so timeout -k 10 300 python scripts/cq_ab.py --rounds 2 --spheres 10000 > $OUT/$v.log 2>&1 || { tail $OUT/$v.log; exit 1; }
  echo "$v $(grep best_ms $OUT/$v.log)"
done
