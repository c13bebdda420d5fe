#!/bin/bash
# Round 4: the one-frame split at N = 8 (per-shard emulation, K = 20, copy
# stream, 16 hardware queues) around the bench's defaults; and the bounce
# launch of the timed shape ALONE under the kernel trace (its mean must agree
# with the counter pass's exclusive time, the roofline's kernel_ms).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04g
mkdir -p "$OUT"
step() {
    local name=$1 lim=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; grep '^{' "$OUT/$name.log" | cut -c1-400 | tail -n 3
    if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step prof_exclusive 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_exclusive" -o run -- python3 bench.py --no-cpu --no-host --pipeline 1 --bounce-blocks 384 --steps 20 --warmup 5
export GPU_MAX_HW_QUEUES=16
S="python3 scripts/shard_times.py --pipeline 8 --steps 5 --copy"
step base_r1 120 $S --batch 4 --worlds 1,8
step base_r2 120 $S --batch 4 --worlds 1,8
step tail1 120 $S --batch 4 --worlds 8 --tail-grid 1
step tail2 120 $S --batch 4 --worlds 8 --tail-grid 2
step blocks512 120 $S --batch 4 --worlds 8 --blocks 512
step blocks640 120 $S --batch 4 --worlds 8 --blocks 640
step blocks256 120 $S --batch 4 --worlds 8 --blocks 256
step b2p12 120 python3 scripts/shard_times.py --pipeline 12 --steps 10 --copy --batch 2 --worlds 8
step b5 120 python3 scripts/shard_times.py --pipeline 8 --steps 4 --copy --batch 5 --worlds 8
step base_r3 120 $S --batch 4 --worlds 1,8

unset GPU_MAX_HW_QUEUES
step gather_overhead 120 env MASTER_ADDR=127.0.0.1 MASTER_PORT=29741 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 python3 scripts/gather_overhead.py
step rccl_tests 200 python -u -m pytest tests/test_bench_launch.py tests/test_gpu_parity.py -m gpu -x -q -k "rccl or shard" --timeout 120 --timeout-method thread
echo done
