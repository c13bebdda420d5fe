#!/bin/bash
# Round 5, first session: the mirt_multi tests, the new bench line (N = 1
# through mirt_multi/RCCL into host memory), the host-link probe, and the
# per-shard emulation of the N-GPU loop (both deliveries).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05a
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
step pytest_multi 600 python -u -m pytest tests/test_multi.py tests/test_bench_launch.py -m gpu -x -v --timeout 200 --timeout-method thread || exit 1
step pytest_parity 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "sharded or double_buffered or bench_launch_plan" || exit 1
step d2h 120 python scripts/d2h_probe.py
step bench 600 python bench.py --steps 20 --warmup 5
grep '^{' $OUT/bench.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ("value","ms_per_step","device_resident_mrays_s","depth1_mrays_s","host_blocking_mrays_s","last_frame_equals_one_context")}, d["roofline"]["frac"], d["cpu_baseline"]["value"])'
step emu_gather 600 python scripts/multi_emulate.py --worlds 1,2,4,8 --delivery gather
step emu_direct 600 python scripts/multi_emulate.py --worlds 1,2,4,8 --delivery host-direct
echo done
