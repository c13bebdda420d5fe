#!/bin/bash
# Round 5, session bd: parity after restricting the lazy fold to one-frame
# launches (accumulation / multi / C loop tests, then the whole suite), the
# N = 8 emulation, and the N = 1 bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05bd
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "gpu suite failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
export GPU_MAX_HW_QUEUES=16
for r in 1 2; do
  timeout -k 10 300 python scripts/multi_emulate.py --worlds 1,8 --delivery host-direct --rounds 1 > $OUT/emu_r$r.log 2>&1 || { echo failed; exit 1; }
  grep pred_job $OUT/emu_r$r.log | python3 -c "
import sys,json
for l in sys.stdin: d=json.loads(l); print('r$r world', d['world'], d['pred_job_mrays_s'])"
done
unset GPU_MAX_HW_QUEUES
timeout -k 10 300 python bench.py --no-cpu --no-host > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -5 $OUT/bench.log; exit 1; }
python3 -c "
import json
t=open('$OUT/bench.log').read(); d=json.loads(t[t.index('{\"metric'):].split('\n')[0])
print('bench', d['value'], d['ms_per_step'], 'dev', d['device_resident_mrays_s'], 'd1', d['depth1_mrays_s'], 'ok', d['last_frame_equals_one_context'])"
