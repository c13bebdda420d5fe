#!/bin/bash
# The GPU suite on the in-tree library (the candidate), then scripts/ab_only.sh:
#   bash scripts/ab_session_quick.sh NAME ab/libmirt_a.so ab/libmirt_b.so [more.so ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/$1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$1/pytest_gpu.log 2>&1
rc=$?
tail -n 2 gpurun_out/$1/pytest_gpu.log
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
bash scripts/ab_only.sh "$@"
