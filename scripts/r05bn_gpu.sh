#!/bin/bash
# Round 5, session bn: the N = 8 per-shard emulation with MORE persistent
# bounce workgroups per launch than the default 384 (512, 640; round 5's
# sweep went down from 384 only), interleaved with 384, two rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05bn
mkdir -p $OUT
for r in 1 2; do
  for bb in 384 512 640; do
    timeout -k 10 300 python scripts/multi_emulate.py --worlds 8 --delivery host-direct --bounce-blocks $bb > $OUT/emu8_bb${bb}_r$r.log 2>&1 || { echo "bb $bb failed"; tail -20 $OUT/emu8_bb${bb}_r$r.log; exit 1; }
    echo "bb $bb round $r: $(grep -o '"rank_ms_per_frame": \[[^]]*\]\|"pred_job_mrays_s": [0-9.]*' $OUT/emu8_bb${bb}_r$r.log | tr '\n' ' ')"
  done
done
