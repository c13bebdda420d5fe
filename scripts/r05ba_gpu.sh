#!/bin/bash
# Round 5, session ba: does the lazy fold cost the N > 1 split? Eager vs lazy
# builds, per-shard emulation at N = 2 and 8, host-direct, interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05ba
mkdir -p $OUT
export GPU_MAX_HW_QUEUES=16
for r in 1 2; do
  for v in eager lazy; do
    MIRT_LIB=$PWD/ab/libmirt_$v.so timeout -k 10 400 python scripts/multi_emulate.py --worlds 1,2,8 --delivery host-direct --rounds 1 > $OUT/emu_${v}_r$r.log 2>&1 || { echo failed; tail -5 $OUT/emu_${v}_r$r.log; exit 1; }
    grep pred_job $OUT/emu_${v}_r$r.log | python3 -c "
import sys,json
for l in sys.stdin: d=json.loads(l); print('$v r$r world', d['world'], d['pred_job_mrays_s'])"
  done
done
