#!/bin/bash
# Round 5, session ad: 4K / 10k at N = 8 through mirt_multi (emulated per
# shard): schedule sweep (lanes:frames per launch:tail launches), host-direct
# and frames left on the device.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05ad
mkdir -p $OUT
export GPU_MAX_HW_QUEUES=16
timeout -k 10 500 python scripts/multi_emulate.py --workload 4k_10k --worlds 8 --delivery host-direct --rounds 1 --sweep 8:4:0,8:2:0,8:4:2,6:4:0,8:8:0 > $OUT/sweep_direct.log 2>&1 || { echo failed; tail -5 $OUT/sweep_direct.log; exit 1; }
timeout -k 10 300 python scripts/multi_emulate.py --workload 4k_10k --worlds 8 --device-only --rounds 1 --sweep 8:4:0,8:4:2 > $OUT/sweep_dev.log 2>&1 || { echo failed; tail -5 $OUT/sweep_dev.log; exit 1; }
cat $OUT/sweep_direct.log $OUT/sweep_dev.log | grep pred_job | python3 -c "
import sys,json
for l in sys.stdin: d=json.loads(l); print(d['delivery'], 'lanes', d['lanes'], 'per', d['frames_per_launch'], 'tail', d['tail_grid'], d['pred_job_mrays_s'], max(d['rank_ms_per_frame']))"
