#!/bin/bash
# Round 5, session u: which host call blocks the queue-ahead loop (HIP API trace).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05u
mkdir -p $OUT
for qa in 0 1; do
  GPU_MAX_HW_QUEUES=16 timeout -k 10 300 rocprofv3 --hip-trace --stats --output-format csv -d $OUT/trace_qa$qa -o run -- python3 scripts/qa_probe.py $qa > $OUT/probe_qa$qa.log 2>&1 || { echo "qa=$qa failed"; tail -20 $OUT/probe_qa$qa.log; exit 1; }
  grep '"ahead"' $OUT/probe_qa$qa.log | cut -c1-400
done
ls -R $OUT | head
