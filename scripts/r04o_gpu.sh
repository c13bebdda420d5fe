#!/bin/bash
# Round 4: the solo drain (the last ray of a bounce wave walked by all 16 of
# its quads). GPU suite on the in-tree build (solo on), bounce stats of one
# launch and of a 1/8 shard, the blocking frame, the 8-shard emulation, and
# the A/B against the same tree without it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=r04o
OUT=gpurun_out/$T
mkdir -p $OUT
step() {
    local name=$1 lim=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; grep -E '^\{|passed|failed' "$OUT/$name.log" | cut -c1-700 | tail -n 3
    if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
for lib in nosolo solo; do
  step bstats_$lib 120 env MIRT_LIB=ab/libmirt_$lib.so python scripts/bounce_stats.py --spheres 10000 --shards 1,8
  step blocking_$lib 120 env MIRT_LIB=ab/libmirt_$lib.so python scripts/blocking_frame.py
done
timeout -k 10 400 python scripts/ab_libs.py ab/libmirt_nosolo.so ab/libmirt_solo.so --rounds 3 --steps 20 > $OUT/ab_10k.log 2>&1 || exit 1
timeout -k 10 400 python scripts/ab_libs.py ab/libmirt_nosolo.so ab/libmirt_solo.so --rounds 2 --steps 20 --workload 1080p_100k > $OUT/ab_100k.log 2>&1 || exit 1
grep BEST $OUT/ab_*.log
export GPU_MAX_HW_QUEUES=16
for lib in nosolo solo; do
  step emu8_$lib 200 env MIRT_LIB=ab/libmirt_$lib.so python3 scripts/shard_times.py --pipeline 8 --steps 5 --copy --batch 4 --worlds 1,8 --tail-grid 2
done
echo done
