#!/bin/bash
# Pipelined bench.py value for each OPTION=VALUE, interleaved rounds:
#   scripts/opt_sweep.sh <tag> <rounds> "5=16" "5=32" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1; R=$2; shift 2
mkdir -p "$OUT"
for r in $(seq 1 "$R"); do
  for o in "$@"; do
    timeout -k 10 120 python bench.py --no-cpu --no-host --steps 100 --opt "$o" > "$OUT/b_${o/=/_}_$r.log" 2>&1 || exit $?
    v=$(grep -o '"value": [0-9.]*' "$OUT/b_${o/=/_}_$r.log" | head -1)
    k=$(grep -o '"kernel_ms": [0-9.]*' "$OUT/b_${o/=/_}_$r.log" | head -1)
    echo "$o round $r $v $k" | tee -a "$OUT/summary.txt"
  done
done
