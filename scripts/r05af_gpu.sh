#!/bin/bash
# Round 5, session af: the multi tests with the copy-stream modes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05af
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_multi.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_multi.log 2>&1 || { echo "multi tests failed"; tail -30 $OUT/pytest_multi.log; exit 1; }
tail -1 $OUT/pytest_multi.log
