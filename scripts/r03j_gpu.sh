#!/bin/bash
# Round 3: bounce workgroups per launch x refill threshold at the driver's
# K = 20 on the committed tree (octant-grouped first bounces), 3 rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r03j
mkdir -p "$OUT"
for rep in 1 2 3; do
  for bb in 320 384 448; do
    for thr in 16 20 24; do
      timeout -k 10 120 python bench.py --no-cpu --no-host --steps 20 --warmup 5 --bounce-blocks $bb --opt 5=$thr > "$OUT/run.log" 2>&1 || { echo "rc=$? bb=$bb thr=$thr"; tail -3 "$OUT/run.log"; exit 1; }
      v=$(grep '^{' "$OUT/run.log" | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['value'])")
      echo "rep=$rep bb=$bb thr=$thr value=$v" | tee -a "$OUT/sweep.txt"
    done
  done
done
echo done
