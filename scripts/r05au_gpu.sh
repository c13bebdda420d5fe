#!/bin/bash
# Round 5, session au: the short last row block copied as a one-row 2D copy
# (was a 1D copy after the strided one): parity, then N = 2 / 4 with 16-, 32-
# and 64-row blocks (whose last block is short) against 8.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05au
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_multi.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_multi.log 2>&1 || { echo "multi tests failed"; tail -30 $OUT/pytest_multi.log; exit 1; }
tail -1 $OUT/pytest_multi.log
export GPU_MAX_HW_QUEUES=16
for rb in 8 16 32 64; do
  timeout -k 10 300 python scripts/multi_emulate.py --worlds 2,4 --delivery host-direct --rounds 1 --row-block $rb > $OUT/rb$rb.log 2>&1 || { echo failed; tail -5 $OUT/rb$rb.log; exit 1; }
done
cat $OUT/rb*.log | grep pred_job | python3 -c "
import sys,json
for l in sys.stdin: d=json.loads(l); print('world', d['world'], 'rb', d['row_block'], d['pred_job_mrays_s'], [round(x,3) for x in d['rank_ms_per_frame']])"
