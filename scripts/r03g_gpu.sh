#!/bin/bash
# Round 3: the multi-GPU defaults (8 ctxs per rank, 16 hardware queues) with
# the gather's stream priced in; the published benchmark-mode sweep with the
# BVH loop checked at every point.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r03g
mkdir -p "$OUT"
step() {
    local name=$1 lim=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -n 1 "$OUT/$name.log" | cut -c1-300
    if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step p8_b4_copy_q16 300 env GPU_MAX_HW_QUEUES=16 python3 scripts/shard_times.py --pipeline 8 --batch 4 --steps 5 --copy
step p8_b4_copy_q8 300 env GPU_MAX_HW_QUEUES=8 python3 scripts/shard_times.py --pipeline 8 --batch 4 --steps 5 --copy
step p8_b4_q16 300 env GPU_MAX_HW_QUEUES=16 python3 scripts/shard_times.py --pipeline 8 --batch 4 --steps 5
step p8_b2_copy_q16 300 env GPU_MAX_HW_QUEUES=16 python3 scripts/shard_times.py --pipeline 8 --batch 2 --steps 10 --copy
step p8_b1_copy_q16 300 env GPU_MAX_HW_QUEUES=16 python3 scripts/shard_times.py --pipeline 8 --batch 1 --steps 20 --copy
step p8_b4_4k_copy_q16 300 env GPU_MAX_HW_QUEUES=16 python3 scripts/shard_times.py --pipeline 8 --batch 4 --steps 5 --copy --width 3840 --height 2160
step p8_b2_4k_copy_q16 300 env GPU_MAX_HW_QUEUES=16 python3 scripts/shard_times.py --pipeline 8 --batch 2 --steps 10 --copy --width 3840 --height 2160
step p8_4k1m_copy_q16 600 env GPU_MAX_HW_QUEUES=16 python3 scripts/shard_times.py --pipeline 8 --steps 20 --copy --width 3840 --height 2160 --scene bench --spheres 1000000 --spp 4
step bench_mode 900 python -u scripts/bench_mode_published.py --out "$OUT/r03_bench_mode"
echo done
