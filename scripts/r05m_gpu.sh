#!/bin/bash
# Round 5, session m: one issuing thread per rank in mirt_multi -- the multi
# tests, the C callers over N ranks, the host cost per launch, the bench line
# and the N = 8 emulation.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05m
mkdir -p "$OUT"
step() {
    local name=$1 lim=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -n 3 "$OUT/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return $rc
}
step pytest_multi 600 python -u -m pytest tests/test_multi.py tests/test_c_dropin.py tests/test_bench_launch.py -m gpu -x -v --timeout 200 --timeout-method thread || exit 1
GPU_MAX_HW_QUEUES=16 step host_issue 300 python scripts/host_issue.py
grep '^{' $OUT/host_issue.log
step bench 600 python bench.py --steps 20 --warmup 5 --no-cpu
grep '^{' $OUT/bench.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ("value","ms_per_step","device_resident_mrays_s","depth1_mrays_s","host_blocking_mrays_s","last_frame_equals_one_context","host_enqueue_ms_per_launch")})'
step emu8 600 python scripts/multi_emulate.py --worlds 1,8 --delivery host-direct --rounds 3
grep -h pred_job $OUT/emu8.log
echo done
