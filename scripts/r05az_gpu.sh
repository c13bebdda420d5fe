#!/bin/bash
# Round 5, session az: per-shard emulation at N = 1 / 2 / 4 / 8 through
# mirt_multi after the 2D D2H and the lazy fold (host-direct, the bench's
# schedule), two rounds; 4K / 10k at 1 and 8.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05az
mkdir -p $OUT
export GPU_MAX_HW_QUEUES=16
for r in 1 2; do
  timeout -k 10 500 python scripts/multi_emulate.py --worlds 1,2,4,8 --delivery host-direct --rounds 1 > $OUT/emu_r$r.log 2>&1 || { echo failed; tail -5 $OUT/emu_r$r.log; exit 1; }
done
timeout -k 10 500 python scripts/multi_emulate.py --workload 4k_10k --worlds 1,8 --delivery host-direct --rounds 1 > $OUT/emu_4k.log 2>&1 || { echo failed; tail -5 $OUT/emu_4k.log; exit 1; }
cat $OUT/*.log | grep pred_job | python3 -c "
import sys,json
for l in sys.stdin: d=json.loads(l); print(d['workload'], 'world', d['world'], 'lanes', d['lanes'], 'per', d['frames_per_launch'], d['pred_job_mrays_s'])"
