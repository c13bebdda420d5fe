#!/bin/bash
# Round 5, session b: rank 0's slabs in place (no RCCL at n = 1), the bench
# line, and the per-shard emulation: gather / host-direct (2D and per-block
# copies) / device-only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05b
mkdir -p "$OUT"
step() {
    local name=$1 lim=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -n 2 "$OUT/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return $rc
}
step pytest_multi 600 python -u -m pytest tests/test_multi.py tests/test_bench_launch.py -m gpu -x -q --timeout 200 --timeout-method thread || exit 1
step pytest_parity 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "sharded or double_buffered or bench_launch_plan" || exit 1
step bench 600 python bench.py --steps 20 --warmup 5 --no-cpu
grep '^{' $OUT/bench.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ("value","ms_per_step","device_resident_mrays_s","depth1_mrays_s","host_blocking_mrays_s","last_frame_equals_one_context")})'
step emu_dev 600 python scripts/multi_emulate.py --worlds 1,8 --device-only
step emu_gather 600 python scripts/multi_emulate.py --worlds 1,8 --delivery gather
step emu_direct 600 python scripts/multi_emulate.py --worlds 8 --delivery host-direct
step emu_direct1 600 python scripts/multi_emulate.py --worlds 8 --delivery host-direct --direct-copy 1
grep -h pred_job $OUT/emu_*.log | python3 -c 'import json,sys
for l in sys.stdin: d=json.loads(l); print(d["delivery"], d["direct_copy"], d["world"], d["pred_job_mrays_s"], d["rank_ms_per_frame"])'
echo done
