#!/bin/bash
# Round 3: full GPU suite after the eight-wide walk was removed (plus the
# one-rank RCCL gather test), the smoke, the driver's bench command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r03n
mkdir -p "$OUT"
echo "GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES-unset} HIP_VISIBLE_DEVICES=${HIP_VISIBLE_DEVICES-unset}" | tee "$OUT/env.txt"
step() {
    local name=$1 lim=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -n 3 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --steps 20 --warmup 5
echo done
