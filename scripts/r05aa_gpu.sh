#!/bin/bash
# Round 5, session aa: queue-ahead with COPY_STREAM 2 (a context's next launch
# waits for its last launch's KERNELS only; the D2H runs on the copy stream)
# against the base loop, N = 1 into host memory, 8 and 16 queues; then the
# multi tests with that mode through the env switch of the test.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05aa
mkdir -p $OUT
for r in 1 2; do
  for q in 8 16; do
    for v in "0 0" "1 2"; do
      set -- $v
      GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python3 scripts/qa_probe.py $1 $2 > $OUT/probe_q${q}_qa$1_cs$2_r$r.log 2>&1 || { echo "failed"; tail -5 $OUT/probe_q${q}_qa$1_cs$2_r$r.log; exit 1; }
      grep '"ahead"' $OUT/probe_q${q}_qa$1_cs$2_r$r.log | tail -1 | python3 -c "
import sys,json
d=json.loads(sys.stdin.read()); e=sorted(d['enqueue_ms']); print('q=$q qa=$1 cs=$2 r=$r', d['mrays_s'], 'enqueue median', e[len(e)//2], 'max', e[-1])"
    done
  done
done
