#!/bin/bash
# Pipelined bench.py value per (workload, pipeline contexts, bounce workgroups = MIRT_OPT_BOUNCE_BLOCKS):
#   scripts/blocks_sweep.sh <tag> <rounds> "<workloads>" "<pipelines>" "<blocks>"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1; R=$2; WLS=$3; PIPES=$4; BLOCKS=$5
mkdir -p "$OUT"
for r in $(seq 1 "$R"); do
  for wl in $WLS; do for p in $PIPES; do for b in $BLOCKS; do
    f="$OUT/b_${wl}_p${p}_b${b}_$r.log"
    timeout -k 10 180 python bench.py --no-cpu --no-host --steps 100 --workload "$wl" --pipeline "$p" --opt "9=$b" > "$f" 2>&1 || exit $?
    v=$(grep -o '"value": [0-9.]*' "$f" | head -1)
    k=$(grep -o '"kernel_ms": [0-9.]*' "$f" | head -1)
    echo "$wl pipeline $p blocks $b round $r $v $k" | tee -a "$OUT/summary.txt"
  done; done; done
done
