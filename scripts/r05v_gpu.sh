#!/bin/bash
# Round 5, session v: queue-ahead vs base with the runtime's SDMA engines off
# (HSA_ENABLE_SDMA=0: copies run as blit kernels on the stream's compute
# queue, so a copy stream's wait on a kernel stream is a queue barrier, not a
# host wait), N = 1 frame loop to host memory, fresh processes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05v
mkdir -p $OUT
for r in 1 2; do
  for sd in 1 0; do
    for qa in 0 1; do
      HSA_ENABLE_SDMA=$sd GPU_MAX_HW_QUEUES=16 timeout -k 10 120 python3 scripts/qa_probe.py $qa > $OUT/probe_sdma${sd}_qa${qa}_r$r.log 2>&1 || { echo "failed"; tail -5 $OUT/probe_sdma${sd}_qa${qa}_r$r.log; exit 1; }
      grep '"ahead"' $OUT/probe_sdma${sd}_qa${qa}_r$r.log | tail -1 | python3 -c "
import sys,json
d=json.loads(sys.stdin.read()); e=sorted(d['enqueue_ms']); print('sdma=$sd qa=$qa r=$r', d['mrays_s'], 'enqueue median', e[len(e)//2], 'max', e[-1])"
    done
  done
done
