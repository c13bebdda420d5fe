#!/bin/bash
# Round 5, session g: the continuation queue with one consumer wave per CU
# (parity + the blocking call), the bench line with the primed loop, the
# per-shard emulation at N = 8 (both deliveries, device-only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05g
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
step pytest_cq 400 python -u -m pytest tests/test_cont_queue.py -m gpu -x -v --timeout 200 --timeout-method thread || exit 1
step cq_ab 400 python scripts/cq_ab.py --rounds 3
grep '"best_ms"' $OUT/cq_ab.log
step bench 600 python bench.py --steps 20 --warmup 5 --no-cpu
grep '^{' $OUT/bench.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ("value","ms_per_step","device_resident_mrays_s","depth1_mrays_s","host_blocking_mrays_s","last_frame_equals_one_context")})'
step emu_direct 600 python scripts/multi_emulate.py --worlds 1,8 --delivery host-direct
step emu_gather 600 python scripts/multi_emulate.py --worlds 8 --delivery gather
step emu_dev 600 python scripts/multi_emulate.py --worlds 8 --device-only
grep -h pred_job $OUT/emu_*.log | python3 -c 'import json,sys
for l in sys.stdin: d=json.loads(l); print(d["delivery"], d["world"], d["pred_job_mrays_s"], d["rank_ms_per_frame"])'
echo done
