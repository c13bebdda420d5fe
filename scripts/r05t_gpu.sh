#!/bin/bash
# Round 5, session t: MIRT_MULTI_QUEUE_AHEAD with one copy stream per context
# and enough hardware queues (N = 1: 4 contexts + 4 copy streams; 8 and 16
# queues), against the default at the same queue counts.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05t
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_multi.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_multi.log 2>&1 || { echo "multi tests failed"; tail -30 $OUT/pytest_multi.log; exit 1; }
tail -1 $OUT/pytest_multi.log
for r in 1 2; do
  for q in 8 16; do
    for qa in 0 1; do
      GPU_MAX_HW_QUEUES=$q timeout -k 10 240 python bench.py --no-cpu --no-host --queue-ahead $qa > $OUT/bench_q${q}_qa${qa}_r$r.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench_q${q}_qa${qa}_r$r.log; exit 1; }
      python3 -c "
import json,sys
t=open('$OUT/bench_q${q}_qa${qa}_r$r.log').read(); d=json.loads(t[t.index('{\"metric'):].split('\n')[0])
print('q=$q qa=$qa r=$r', d['value'], d['ms_per_step'], d['device_resident_mrays_s'], d['depth1_mrays_s'], d['last_frame_equals_one_context'])"
    done
  done
done
