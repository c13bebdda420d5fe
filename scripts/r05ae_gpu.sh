#!/bin/bash
# Round 5, session ae: the interleave block (rows per shard block) at N = 8,
# emulated per shard, host-direct, 1080p / 10k and 4K / 10k.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05ae
mkdir -p $OUT
export GPU_MAX_HW_QUEUES=16
for wl in 1080p_10k 4k_10k; do
  for rb in 8 16 32 64; do
    timeout -k 10 300 python scripts/multi_emulate.py --workload $wl --worlds 8 --delivery host-direct --rounds 1 --row-block $rb > $OUT/emu_${wl}_rb$rb.log 2>&1 || { echo failed; tail -5 $OUT/emu_${wl}_rb$rb.log; exit 1; }
    grep pred_job $OUT/emu_${wl}_rb$rb.log | python3 -c "
import sys,json
for l in sys.stdin: d=json.loads(l); print('$wl rb', d['row_block'], d['pred_job_mrays_s'], d['rank_ms_per_frame'])"
  done
done
