#!/bin/bash
# Round 5, session bh: N = 8 (and 1, 2) emulation: the ordered batch fold
# (base) vs batches left pending (lazyb) vs pending + launches completing in
# issue order by a stream barrier (lazyord); three interleaved rounds; then
# the multi parity tests on lazyord.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05bh
mkdir -p $OUT
MIRT_LIB=$PWD/ab/libmirt_lazyord.so timeout -k 10 300 python -u -m pytest tests/test_multi.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_multi_lazyord.log 2>&1 || { echo "multi tests failed"; tail -30 $OUT/pytest_multi_lazyord.log; exit 1; }
tail -1 $OUT/pytest_multi_lazyord.log
export GPU_MAX_HW_QUEUES=16
for r in 1 2 3; do
  for v in base lazyb lazyord; do
    MIRT_LIB=$PWD/ab/libmirt_$v.so timeout -k 10 300 python scripts/multi_emulate.py --worlds 8,2 --delivery host-direct --rounds 1 > $OUT/emu_${v}_r$r.log 2>&1 || { echo failed; tail -5 $OUT/emu_${v}_r$r.log; exit 1; }
    grep pred_job $OUT/emu_${v}_r$r.log | python3 -c "
import sys,json
for l in sys.stdin: d=json.loads(l); print('$v r$r world', d['world'], d['pred_job_mrays_s'])"
  done
done
