#!/bin/bash
# Round 3: size-adaptive batched leaf gates (MIRT_OPT_LEAF_BATCH, auto = on for
# trees past the L2): full GPU suite, then 4K/1M with auto vs forced off, and
# the headline bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r03u
mkdir -p "$OUT"
step() {
    local name=$1 lim=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-400
    if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
for r in 1 2; do
    step bench_4k1m_auto_$r 300 python bench.py --steps 20 --warmup 5 --no-cpu --no-host --workload 4k_1m_4spp
    step bench_4k1m_off_$r 300 python bench.py --steps 20 --warmup 5 --no-cpu --no-host --workload 4k_1m_4spp --opt 14=0
done
step bench 600 python bench.py --steps 20 --warmup 5
echo done
