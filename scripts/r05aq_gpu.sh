#!/bin/bash
# Round 5, session aq: the host-direct copy shape issued as mirt_multi issues it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05aq
mkdir -p $OUT
for w in 8 4 2; do
  timeout -k 10 120 python scripts/d2h2d_probe.py --world $w > $OUT/d2h2d_w$w.log 2>&1 || { echo failed; tail -5 $OUT/d2h2d_w$w.log; exit 1; }
  grep world $OUT/d2h2d_w$w.log
done
