#!/bin/bash
# Round 4: next-node prefetch A/B (trace.h NodePf) at 5 and 4 bounce waves per SIMD.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=r04c
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 || { tail -20 gpurun_out/$T/pytest.log; exit 1; }
tail -n 2 gpurun_out/$T/pytest.log
L="ab/libmirt_base.so ab/libmirt_pf4w4.so ab/libmirt_pf4w5.so ab/libmirt_w4.so"
timeout -k 10 400 python scripts/ab_libs.py $L --rounds 2 --steps 20 > gpurun_out/$T/ab_10k.log 2>&1 || exit 1
timeout -k 10 400 python scripts/ab_libs.py $L --rounds 2 --steps 20 --workload 1080p_100k > gpurun_out/$T/ab_100k.log 2>&1 || exit 1
grep BEST gpurun_out/$T/ab_*.log
timeout -k 10 120 python scripts/blocking_frame.py > gpurun_out/$T/blocking.log 2>&1 || exit 1
tail -1 gpurun_out/$T/blocking.log
