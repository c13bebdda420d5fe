#!/bin/bash
# Round 5, session bc: eager vs lazy fold at N = 8 (emulated, host-direct),
# four interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05bc
mkdir -p $OUT
export GPU_MAX_HW_QUEUES=16
for r in 1 2 3 4; do
  for v in eager lazy; do
    MIRT_LIB=$PWD/ab/libmirt_$v.so timeout -k 10 300 python scripts/multi_emulate.py --worlds 8 --delivery host-direct --rounds 1 > $OUT/emu_${v}_r$r.log 2>&1 || { echo failed; tail -5 $OUT/emu_${v}_r$r.log; exit 1; }
    grep pred_job $OUT/emu_${v}_r$r.log | python3 -c "
import sys,json
for l in sys.stdin: d=json.loads(l); print('$v r$r world', d['world'], d['pred_job_mrays_s'], max(d['rank_ms_per_frame']), min(d['rank_ms_per_frame']))"
  done
done
