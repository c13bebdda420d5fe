#!/bin/bash
# Round 3: the one-frame split at the driver's step count (K = 20 frames per
# rank, so 20 / batch launches), frames per launch 1 / 2 / 4, per shard on
# one GPU; and the other workloads' bench lines with the new timed loop.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r03d
mkdir -p "$OUT"
step() {
    local name=$1 lim=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -n 1 "$OUT/$name.log" | cut -c1-300
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
for rep in 1 2; do
  step k20_b1_r$rep 300 python3 scripts/shard_times.py --pipeline 4 --batch 1 --steps 20
  step k20_b2_r$rep 300 python3 scripts/shard_times.py --pipeline 4 --batch 2 --steps 10
  step k20_b4_r$rep 300 python3 scripts/shard_times.py --pipeline 4 --batch 4 --steps 5
done
step k20_4k_b1 300 python3 scripts/shard_times.py --pipeline 4 --batch 1 --steps 20 --width 3840 --height 2160
step k20_4k_b2 300 python3 scripts/shard_times.py --pipeline 4 --batch 2 --steps 10 --width 3840 --height 2160
step k20_4k_b4 300 python3 scripts/shard_times.py --pipeline 4 --batch 4 --steps 5 --width 3840 --height 2160
step bench_k20 300 python bench.py --no-cpu --no-host --steps 20 --warmup 5
step bench_k20_acc 300 python bench.py --no-cpu --no-host --steps 20 --warmup 5 --accumulate
for wl in 1080p_100k 4k_10k 4k_1m_4spp; do
  step bench_$wl 600 python bench.py --no-cpu --no-host --steps 20 --warmup 5 --workload $wl
done
echo done
