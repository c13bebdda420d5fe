#!/bin/bash
# Round 4: the blocking call (a frame alone) against the bounce pass's
# refill threshold (MIRT_OPT_BOUNCE_THRESHOLD, 5) and the quad drain (11).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04aj
mkdir -p $OUT
for r in 1 2; do
  for o in "5=20" "5=8" "5=12" "5=28" "5=40" "5=56" "11=0"; do
    n=$(echo $o | tr '=' '_')
    timeout -k 10 120 python scripts/blocking_frame.py --opt $o > $OUT/blocking_${n}_r$r.log 2>&1 || { tail -5 $OUT/blocking_${n}_r$r.log; exit 1; }
    echo "$o r$r $(tail -1 $OUT/blocking_${n}_r$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["pinned_ms"], d["pageable_ms"], d["kernels_ms"], d["frames_equal"])')"
  done
done
