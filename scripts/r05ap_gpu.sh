#!/bin/bash
# Round 5, session ap: host-direct delivery by a copy kernel into the mapped
# frame (DIRECT_COPY 2) -- parity, then the per-shard emulation at N = 2 / 4
# / 8 against the strided DMA (0) and no delivery, two rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05ap
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_multi.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_multi.log 2>&1 || { echo "multi tests failed"; tail -30 $OUT/pytest_multi.log; exit 1; }
tail -1 $OUT/pytest_multi.log
export GPU_MAX_HW_QUEUES=16
for r in 1 2; do
  for dc in 0 2; do
    timeout -k 10 400 python scripts/multi_emulate.py --worlds 2,4,8 --delivery host-direct --direct-copy $dc --rounds 1 > $OUT/dc${dc}_r$r.log 2>&1 || { echo failed; tail -5 $OUT/dc${dc}_r$r.log; exit 1; }
  done
done
timeout -k 10 400 python scripts/multi_emulate.py --worlds 1 --delivery host-direct --direct-copy 2 --rounds 1 > $OUT/dc2_w1.log 2>&1 || { echo failed; exit 1; }
for f in $OUT/dc*.log; do grep pred_job $f | python3 -c "
import sys,json
for l in sys.stdin: d=json.loads(l); print('$(basename $f)', 'world', d['world'], 'dc', d['direct_copy'], d['pred_job_mrays_s'])"; done
