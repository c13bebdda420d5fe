#!/bin/bash
# Round 4: the blocking frame by destination (incl. zero-copy), and the
# 8-GPU one-frame split emulated per shard (the bench's N > 1 defaults) with
# its kernel trace and the bounce tail of a 1/8 shard.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04e
mkdir -p "$OUT"
step() {
    local name=$1 lim=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-600
    if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step blocking 120 python scripts/blocking_frame.py
step bstats_shard8 120 python scripts/bounce_stats.py --spheres 10000 --shards 1,8
export GPU_MAX_HW_QUEUES=16
step p8_b4_copy 300 python3 scripts/shard_times.py --pipeline 8 --batch 4 --steps 5 --copy --worlds 1,8
step trace_p8 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_p8" -o run -- python3 scripts/shard_times.py --pipeline 8 --batch 4 --steps 5 --copy --worlds 8
echo done
