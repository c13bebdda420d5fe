#!/bin/bash
# Round 5, session r: N = 1 lanes x hardware queues, frames to host memory
# (the headline's loop) -- does a fifth / sixth lane hide the per-lane D2H and
# host turnaround that cost the host-inclusive loop ~3% against device-resident?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05r
mkdir -p $OUT
timeout -k 10 600 python scripts/n1_sweep.py --lanes 4,5,6 --queues 8,16 --steps 20 --device-only 0 > $OUT/n1_lanes.log 2>&1; rc=$?
grep -v amdgpu.ids $OUT/n1_lanes.log
exit $rc
