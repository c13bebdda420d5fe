#!/bin/bash
# Round 5, session an: frames per launch at N = 4 (2 vs 4) and N = 2 (1 vs 2),
# emulated per shard through mirt_multi, host-direct, three rounds each,
# interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05an
mkdir -p $OUT
export GPU_MAX_HW_QUEUES=16
for r in 1 2 3; do
  timeout -k 10 400 python scripts/multi_emulate.py --worlds 4 --delivery host-direct --rounds 1 --sweep 8:2:0,8:4:0 > $OUT/n4_r$r.log 2>&1 || { echo failed; exit 1; }
  timeout -k 10 400 python scripts/multi_emulate.py --worlds 2 --delivery host-direct --rounds 1 --sweep 8:1:0,8:2:0 > $OUT/n2_r$r.log 2>&1 || { echo failed; exit 1; }
done
cat $OUT/*.log | grep pred_job | python3 -c "
import sys,json,collections
r=collections.defaultdict(list)
for l in sys.stdin: d=json.loads(l); r[(d['world'], d['frames_per_launch'])].append(d['pred_job_mrays_s'])
for k,v in sorted(r.items()): print('world', k[0], 'per', k[1], v)"
