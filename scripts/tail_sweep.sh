#!/bin/bash
# bench.py at the driver's K = 20 with the last T launches of the timed burst
# on the full bounce grid (--tail-grid T), rounds interleaved:
#   bash scripts/tail_sweep.sh <tag> <rounds> "<workloads>" "<tails>"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1; R=$2; WLS=$3; TAILS=$4
mkdir -p "$OUT"
for r in $(seq 1 "$R"); do
  for wl in $WLS; do for t in $TAILS; do
    f="$OUT/t_${wl}_tail${t}_$r.log"
    timeout -k 10 180 python bench.py --no-cpu --no-host --steps 20 --warmup 5 --workload "$wl" --tail-grid "$t" > "$f" 2>&1 || exit $?
    v=$(grep -o '"value": [0-9.]*' "$f" | head -1)
    k=$(grep -o '"kernel_ms": [0-9.]*' "$f" | head -1)
    echo "$wl tail $t round $r $v $k" | tee -a "$OUT/summary.txt"
  done; done
done
