#!/bin/bash
# Round 5, session ab: N = 8 per-shard emulation (host-direct, 4 frames per
# launch), persistent bounce workgroups per launch x lanes -- 8 lanes at 384
# workgroups ask the CU for 12 bounce workgroups' LDS where 6 fit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05ab
mkdir -p $OUT
export GPU_MAX_HW_QUEUES=16
for bb in 384 192 256 128; do
  timeout -k 10 300 python scripts/multi_emulate.py --worlds 8 --delivery host-direct --bounce-blocks $bb --sweep 8:4:0,6:4:0,12:4:0 > $OUT/emu8_bb$bb.log 2>&1 || { echo "bb=$bb failed"; tail -5 $OUT/emu8_bb$bb.log; exit 1; }
  grep pred_job $OUT/emu8_bb$bb.log | python3 -c "
import sys,json
for l in sys.stdin: d=json.loads(l); print('bb', d['bounce_blocks'], 'lanes', d['lanes'], 'per', d['frames_per_launch'], d['pred_job_mrays_s'])"
done
