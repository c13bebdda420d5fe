#!/bin/bash
# Round 5, session be (after the lazy-fold policy): is the N = 8 emulation's drop (15.3-15.5 -> 13.2-14.1
# Grays/s) the library's? The build of commit ad518b0 (old) against the
# current one (cur), interleaved, per-shard emulation at N = 8 and 2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05be
mkdir -p $OUT
export GPU_MAX_HW_QUEUES=16
for r in 1 2 3; do
  for v in old cur; do
    MIRT_LIB=$PWD/ab/libmirt_$v.so timeout -k 10 400 python scripts/multi_emulate.py --worlds 8 --delivery host-direct --rounds 1 > $OUT/emu_${v}_r$r.log 2>&1 || { echo failed; tail -5 $OUT/emu_${v}_r$r.log; exit 1; }
    grep pred_job $OUT/emu_${v}_r$r.log | python3 -c "
import sys,json
for l in sys.stdin: d=json.loads(l); print('$v r$r world', d['world'], d['pred_job_mrays_s'])"
  done
done
