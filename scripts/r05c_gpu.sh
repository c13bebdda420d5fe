#!/bin/bash
# Round 5, session c: the N = 1 loop through mirt_multi over lanes / queues /
# delivery / steps, each in a fresh process.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05c
mkdir -p "$OUT"
timeout -k 10 600 python scripts/n1_sweep.py --lanes 4,8 --queues 4,16 --steps 20,100 > $OUT/n1_sweep.log 2>&1; rc=$?
cat $OUT/n1_sweep.log; exit $rc
