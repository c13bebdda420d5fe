#!/bin/bash
# Round 3: benchmark mode at the published sphere counts (1K .. 100M), and
# the one-frame split with RCCL's stream priced against the hardware queues.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r03f
mkdir -p "$OUT"
step() {
    local name=$1 lim=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-400
    if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step bench_mode 900 python -u scripts/bench_mode_published.py --out "$OUT/r03_bench_mode"
step k20_b4_copy_q4 300 python3 scripts/shard_times.py --pipeline 4 --batch 4 --steps 5 --copy
step k20_b4_copy_q8 300 env GPU_MAX_HW_QUEUES=8 python3 scripts/shard_times.py --pipeline 4 --batch 4 --steps 5 --copy
step k20_b4_q8 300 env GPU_MAX_HW_QUEUES=8 python3 scripts/shard_times.py --pipeline 4 --batch 4 --steps 5
step k20_b2_p8_q8 300 env GPU_MAX_HW_QUEUES=8 python3 scripts/shard_times.py --pipeline 8 --batch 2 --steps 10
step k20_b4_p8_q8 300 env GPU_MAX_HW_QUEUES=8 python3 scripts/shard_times.py --pipeline 8 --batch 4 --steps 5
step k20_b1_p8_q8 300 env GPU_MAX_HW_QUEUES=8 python3 scripts/shard_times.py --pipeline 8 --batch 1 --steps 20
echo done
