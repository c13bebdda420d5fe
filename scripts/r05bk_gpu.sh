#!/bin/bash
# Round 5, session bk: the N = 8 per-shard emulation with interleave blocks
# finer than 8 rows (4, 2), interleaved with the default 8 (balance vs the
# camera packets' coherence: a slab's 8-row packet then spans 2 / 4 blocks).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05bk
mkdir -p $OUT
for r in 1 2; do
  for rb in 8 4 2; do
    timeout -k 10 300 python scripts/multi_emulate.py --worlds 8 --delivery host-direct --row-block $rb > $OUT/emu8_rb${rb}_r$r.log 2>&1 || { echo "rb $rb failed"; tail -20 $OUT/emu8_rb${rb}_r$r.log; exit 1; }
    echo "rb $rb round $r: $(grep -o '"rank_ms_per_frame": \[[^]]*\]\|"pred_job_mrays_s": [0-9.]*' $OUT/emu8_rb${rb}_r$r.log | tr '\n' ' ')"
  done
done
