#!/bin/bash
# Round 3: the one-frame split at N = 8 (K = 20 frames per rank) with larger
# launches: 5 / 10 / 20 frames per launch (the whole timed region in 4 / 2 / 1
# launches per rank), RCCL's stream priced in (--copy), 16 queues.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r03k
mkdir -p "$OUT"
step() {
    local name=$1 lim=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; grep '"world": 8' "$OUT/$name.log" | cut -c150-400
    if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
export GPU_MAX_HW_QUEUES=16
step p4_b5 300 python3 scripts/shard_times.py --worlds 4,8 --pipeline 4 --batch 5 --steps 4 --copy
step p8_b5 300 python3 scripts/shard_times.py --worlds 4,8 --pipeline 8 --batch 5 --steps 4 --copy
step p2_b10_bb640 300 python3 scripts/shard_times.py --worlds 4,8 --pipeline 2 --batch 10 --steps 2 --copy --blocks 640
step p2_b10_bb384 300 python3 scripts/shard_times.py --worlds 4,8 --pipeline 2 --batch 10 --steps 2 --copy --blocks 384
step p1_b20_full 300 python3 scripts/shard_times.py --worlds 4,8 --pipeline 1 --batch 20 --steps 1 --copy --blocks 0
step p8_b4 300 python3 scripts/shard_times.py --worlds 4,8 --pipeline 8 --batch 4 --steps 5 --copy
echo done
