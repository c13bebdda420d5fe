#!/bin/bash
# Round 5, session s: MIRT_MULTI_QUEUE_AHEAD (two launch slots per context,
# copies on per-slot copy streams). Parity of the multi tests first, then the
# N = 1 bench loop with and without it (fresh processes, interleaved), then
# the N = 8 per-shard emulation with and without it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05s
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_multi.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_multi.log 2>&1 || { echo "multi tests failed"; tail -30 $OUT/pytest_multi.log; exit 1; }
tail -1 $OUT/pytest_multi.log
for r in 1 2; do
  for qa in 0 1; do
    timeout -k 10 240 python bench.py --no-cpu --no-host --queue-ahead $qa > $OUT/bench_qa${qa}_r$r.log 2>&1 || { echo "bench qa=$qa failed"; tail -20 $OUT/bench_qa${qa}_r$r.log; exit 1; }
    python3 -c "
import json,sys
t=open('$OUT/bench_qa${qa}_r$r.log').read(); d=json.loads(t[t.index('{\"metric'):].split('\n')[0])
print('qa=$qa r=$r', d['value'], d['ms_per_step'], d['device_resident_mrays_s'], d['depth1_mrays_s'], d['last_frame_equals_one_context'])"
  done
done
for qa in 0 1; do
  GPU_MAX_HW_QUEUES=16 timeout -k 10 400 python scripts/multi_emulate.py --worlds 8 --delivery host-direct --queue-ahead $qa > $OUT/emu8_qa$qa.log 2>&1 || { echo "emu qa=$qa failed"; tail -20 $OUT/emu8_qa$qa.log; exit 1; }
  grep pred_job $OUT/emu8_qa$qa.log | python3 -c "
import sys,json
for l in sys.stdin: d=json.loads(l); print('emu8 qa=$qa', d['pred_job_mrays_s'], d['rank_ms_per_frame'])"
done
