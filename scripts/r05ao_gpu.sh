#!/bin/bash
# Round 5, session ao: what the host-direct copies cost at N = 2 / 4 / 8
# (emulated per shard): one strided 2D copy per rank per frame (direct_copy
# 0), one copy per row block (1), and no delivery (device-only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05ao
mkdir -p $OUT
export GPU_MAX_HW_QUEUES=16
for r in 1 2; do
  timeout -k 10 400 python scripts/multi_emulate.py --worlds 2,4,8 --delivery host-direct --rounds 1 > $OUT/dc0_r$r.log 2>&1 || { echo failed; exit 1; }
  timeout -k 10 400 python scripts/multi_emulate.py --worlds 2,4,8 --delivery host-direct --direct-copy 1 --rounds 1 > $OUT/dc1_r$r.log 2>&1 || { echo failed; exit 1; }
  timeout -k 10 400 python scripts/multi_emulate.py --worlds 2,4,8 --delivery host-direct --device-only --rounds 1 > $OUT/dev_r$r.log 2>&1 || { echo failed; exit 1; }
done
for f in $OUT/*.log; do grep pred_job $f | python3 -c "
import sys,json
for l in sys.stdin: d=json.loads(l); print('$(basename $f)', 'world', d['world'], d['delivery'], 'dc', d['direct_copy'], d['pred_job_mrays_s'])"; done
