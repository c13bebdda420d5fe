#!/bin/bash
# Round 5, session k: the N = 8 schedule in the per-shard emulation,
# host-direct, three rounds per shard (best of three), around the defaults.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05k
mkdir -p "$OUT"
timeout -k 10 900 python scripts/multi_emulate.py --worlds 1 --delivery host-direct --rounds 3 > $OUT/w1.log 2>&1 || { tail $OUT/w1.log; exit 1; }
timeout -k 10 900 python scripts/multi_emulate.py --worlds 8 --delivery host-direct --rounds 3 --sweep 8:4:0,8:4:1,8:4:2,6:4:0,6:4:2,10:4:0,8:3:0 > $OUT/sweep.log 2>&1 || { tail $OUT/sweep.log; exit 1; }
for b in 256 512; do
  timeout -k 10 600 python scripts/multi_emulate.py --worlds 8 --delivery host-direct --rounds 3 --bounce-blocks $b --sweep 8:4:0,8:4:2 > $OUT/bb$b.log 2>&1 || { tail $OUT/bb$b.log; exit 1; }
done
grep -h pred_job $OUT/*.log | python3 -c 'import json,sys
for l in sys.stdin: d=json.loads(l); print(d["world"], d["lanes"], d["frames_per_launch"], d["tail_grid"], d["bounce_blocks"], d["pred_job_mrays_s"], max(d["rank_ms_per_frame"]))'
