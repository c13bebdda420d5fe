#!/bin/bash
# bench.py value at 2..5 device contexts in flight (--pipeline), two rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r02u
for r in 1 2; do for p in 2 3 4 5; do timeout -k 10 120 python bench.py --no-cpu --no-host --steps 100 --pipeline $p > gpurun_out/r02u/p${p}_$r.log 2>&1 || exit $?; echo "pipeline $p round $r $(grep -o '"value": [0-9.]*' gpurun_out/r02u/p${p}_$r.log | head -1)" | tee -a gpurun_out/r02u/summary.txt; done; done
