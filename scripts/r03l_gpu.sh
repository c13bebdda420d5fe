#!/bin/bash
# Round 3: the 8-way one-frame split (K = 20), 4 frames per launch: contexts
# x bounce workgroups per launch, RCCL's stream priced in, 16 queues.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r03l
mkdir -p "$OUT"
export GPU_MAX_HW_QUEUES=16
for cfg in "4 640" "4 1280" "6 384" "8 256" "8 384" "8 640" "12 256" "12 384"; do
  set -- $cfg
  timeout -k 10 120 python3 scripts/shard_times.py --worlds 8 --pipeline $1 --blocks $2 --batch 4 --steps 5 --copy > "$OUT/p$1_bb$2.log" 2>&1 || { echo "rc=$? $cfg"; tail -3 "$OUT/p$1_bb$2.log"; exit 1; }
  echo "p=$1 bb=$2 $(grep -o '"pred_job_mrays_s_no_gather": [0-9.]*' "$OUT/p$1_bb$2.log")" | tee -a "$OUT/sweep.txt"
done
echo done
