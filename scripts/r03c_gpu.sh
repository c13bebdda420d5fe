#!/bin/bash
# Round 3: frames per launch at the driver's step count (K = 20) and at
# K = 100, the bench-path parity tests, and the other workloads' lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r03c
mkdir -p "$OUT"
step() {
    local name=$1 lim=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-400
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step pytest_bench_plan 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 200 --timeout-method thread -k "bench_launch_plan or shared_accumulation"
for rep in 1 2; do
  for b in 1 2 4; do
    step k20_b${b}_r$rep 200 python bench.py --no-cpu --no-host --steps 20 --warmup 5 --batch $b
  done
done
for b in 1 4; do
    step k100_b$b 200 python bench.py --no-cpu --no-host --steps 100 --warmup 5 --batch $b
done
echo done
