#!/bin/bash
# Round 5, session at: the interleave block at N = 2 and 4 (emulated per
# shard, host-direct, the bench's schedule), two rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05at
mkdir -p $OUT
export GPU_MAX_HW_QUEUES=16
for r in 1 2; do
  for rb in 8 16 32 64; do
    timeout -k 10 300 python scripts/multi_emulate.py --worlds 2,4 --delivery host-direct --rounds 1 --row-block $rb > $OUT/rb${rb}_r$r.log 2>&1 || { echo failed; tail -5 $OUT/rb${rb}_r$r.log; exit 1; }
  done
done
cat $OUT/*.log | grep pred_job | python3 -c "
import sys,json,collections
r=collections.defaultdict(list)
for l in sys.stdin: d=json.loads(l); r[(d['world'], d['row_block'])].append((d['pred_job_mrays_s'], [round(x,3) for x in d['rank_ms_per_frame']]))
for k,v in sorted(r.items()): print('world', k[0], 'rb', k[1], v)"
