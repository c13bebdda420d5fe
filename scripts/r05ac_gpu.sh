#!/bin/bash
# Round 5, session ac: the BASELINE 8-GPU configs (4K / 10k, 4K / 1M 4 spp)
# through mirt_multi, per-shard emulation at N = 1 and 8, host-direct.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05ac
mkdir -p $OUT
export GPU_MAX_HW_QUEUES=16
for wl in 4k_10k 4k_1m_4spp; do
  timeout -k 10 500 python scripts/multi_emulate.py --workload $wl --worlds 1,8 --delivery host-direct --rounds 1 > $OUT/emu_$wl.log 2>&1 || { echo "$wl failed"; tail -5 $OUT/emu_$wl.log; exit 1; }
  grep pred_job $OUT/emu_$wl.log | python3 -c "
import sys,json
for l in sys.stdin: d=json.loads(l); print('$wl world', d['world'], 'lanes', d['lanes'], 'per', d['frames_per_launch'], d['pred_job_mrays_s'])"
done
