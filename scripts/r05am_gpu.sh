#!/bin/bash
# Round 5, session am: the per-shard emulation at N = 2 and 4 through
# mirt_multi (host-direct), the bench's schedule and neighbours.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05am
mkdir -p $OUT
export GPU_MAX_HW_QUEUES=16
timeout -k 10 400 python scripts/multi_emulate.py --worlds 1,2,4 --delivery host-direct --rounds 2 > $OUT/emu_default.log 2>&1 || { echo failed; tail -5 $OUT/emu_default.log; exit 1; }
timeout -k 10 400 python scripts/multi_emulate.py --worlds 2 --delivery host-direct --rounds 2 --sweep 8:2:0,8:4:0,4:1:0,6:2:0 > $OUT/emu_n2_sweep.log 2>&1 || { echo failed; tail -5 $OUT/emu_n2_sweep.log; exit 1; }
timeout -k 10 400 python scripts/multi_emulate.py --worlds 4 --delivery host-direct --rounds 2 --sweep 8:2:0,6:4:0,8:8:0 > $OUT/emu_n4_sweep.log 2>&1 || { echo failed; tail -5 $OUT/emu_n4_sweep.log; exit 1; }
cat $OUT/emu_default.log $OUT/emu_n2_sweep.log $OUT/emu_n4_sweep.log | grep pred_job | python3 -c "
import sys,json
for l in sys.stdin: d=json.loads(l); print('world', d['world'], 'lanes', d['lanes'], 'per', d['frames_per_launch'], d['pred_job_mrays_s'])"
