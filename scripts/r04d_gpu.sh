#!/bin/bash
# Round 4: banded blocking frames (all bands' kernels first, then the copies).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=r04d
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { tail -20 gpurun_out/$T/pytest.log; exit 1; }
tail -n 2 gpurun_out/$T/pytest.log
timeout -k 10 120 python scripts/blocking_frame.py > gpurun_out/$T/blocking.log 2>&1 || exit 1
tail -1 gpurun_out/$T/blocking.log
