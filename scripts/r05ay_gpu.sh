#!/bin/bash
# Round 5, session ay: queue-ahead re-measured after the 2D D2H and the lazy
# fold (the starvation seen before came with blit-kernel copies and ordered
# folds): base vs ahead with copies behind the kernels (0), on the copy
# stream (1) and early release (2); 8 and 16 queues, two rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05ay
mkdir -p $OUT
for r in 1 2; do
  for q in 8 16; do
    for v in "0 0" "1 0" "1 1" "1 2"; do
      set -- $v
      GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python3 scripts/qa_probe.py $1 $2 > $OUT/probe_q${q}_qa$1_cs$2_r$r.log 2>&1 || { echo "failed"; tail -5 $OUT/probe_q${q}_qa$1_cs$2_r$r.log; exit 1; }
      grep '"ahead"' $OUT/probe_q${q}_qa$1_cs$2_r$r.log | tail -1 | python3 -c "
import sys,json
d=json.loads(sys.stdin.read()); e=sorted(d['enqueue_ms']); print('q=$q qa=$1 cs=$2 r=$r', d['mrays_s'], 'enqueue median', e[len(e)//2], 'max', e[-1])"
    done
  done
done
