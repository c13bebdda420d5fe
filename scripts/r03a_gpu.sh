#!/bin/bash
# Round 3, first GPU session: profile of the configuration bench.py times
# (4 contexts x 384 bounce workgroups, the driver's --steps 20 --warmup 5)
# and the pipelined one-frame split emulated per shard (scripts/shard_times.py).
# Every GPU step has its own time limit; a fault / abort / timeout ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r03a
mkdir -p "$OUT"
step() {
    local name=$1 lim=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -n 3 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step prof_timed 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_timed" -o run -- \
    python3 bench.py --no-cpu --no-host --steps 20 --warmup 5
step strong_p4_1080p 300 python3 scripts/shard_times.py --pipeline 4 --steps 100
step strong_p3copy_1080p 300 python3 scripts/shard_times.py --pipeline 3 --copy --steps 100
step strong_p4copy_1080p 300 python3 scripts/shard_times.py --pipeline 4 --copy --steps 100
step strong_p4_4k 400 python3 scripts/shard_times.py --pipeline 4 --steps 40 --width 3840 --height 2160
step strong_p4_4k1m 600 python3 scripts/shard_times.py --pipeline 4 --steps 12 --width 3840 --height 2160 \
    --scene bench --spheres 1000000 --spp 4
echo done
