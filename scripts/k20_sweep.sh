#!/bin/bash
# bench.py value at the driver's step count (K=20) and at the default (K=100)
# for several frame-scheduling settings, interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-k20}; mkdir -p "$OUT"
for r in 1 2; do
for K in 20 100; do
for cfg in "--pipeline 4" "--pipeline 3 --bounce-blocks 0"; do
  timeout -k 10 120 python bench.py --steps $K --warmup 5 --no-cpu --no-host $cfg > "$OUT/b.log" 2>&1 || exit 1
  echo "K=$K $cfg round $r $(grep -o '"value": [0-9.]*' "$OUT/b.log" | head -1)" | tee -a "$OUT/summary.txt"
done; done; done
