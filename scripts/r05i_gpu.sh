#!/bin/bash
# Round 5, session i: the continuation queue without cache maintenance
# (relaxed atomics), parity + the blocking call, lane / quad pushes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05i
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_cont_queue.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_cq.log 2>&1 || { tail -20 $OUT/pytest_cq.log; exit 1; }
tail -1 $OUT/pytest_cq.log
timeout -k 10 300 python scripts/cq_ab.py --rounds 3 > $OUT/cq_lane.log 2>&1 || { tail $OUT/cq_lane.log; exit 1; }
cat $OUT/cq_lane.log
MIRT_LIB=$PWD/ab/libmirt_cq_quad.so timeout -k 10 300 python scripts/cq_ab.py --rounds 2 > $OUT/cq_quad.log 2>&1 || { tail $OUT/cq_quad.log; exit 1; }
grep best_ms $OUT/cq_quad.log
