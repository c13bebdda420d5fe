#!/bin/bash
# Round 5, session bf: kernel trace of the N = 8 per-shard emulation
# (host-direct): does the runtime insert blit kernels (copies, fills) into
# the ranks' streams?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05bf
mkdir -p $OUT
export GPU_MAX_HW_QUEUES=16
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 scripts/multi_emulate.py --worlds 8 --delivery host-direct --rounds 1 > $OUT/prof.log 2>&1 || { echo failed; tail -5 $OUT/prof.log; exit 1; }
grep pred_job $OUT/prof.log | cut -c1-300
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/r05bf/prof/run_kernel_stats.csv')))
for r in rows[:12]: print(r['Name'][:70], r['Calls'], r['AverageNs'], r['Percentage'])
PY
