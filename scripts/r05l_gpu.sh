#!/bin/bash
# Round 5, session l: the host cost of one thread issuing N ranks' launches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05l
mkdir -p "$OUT"
GPU_MAX_HW_QUEUES=16 timeout -k 10 600 python scripts/host_issue.py > $OUT/host_issue.log 2>&1; rc=$?
cat $OUT/host_issue.log | grep '^{'; exit $rc
