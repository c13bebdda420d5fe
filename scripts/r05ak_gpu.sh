#!/bin/bash
# Round 5, session ak: the bench-launch GPU tests (incl. the N > 1 rehearsal).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05ak
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_bench_launch.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo failed; tail -30 $OUT/pytest.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $OUT/pytest.log | tail -4
