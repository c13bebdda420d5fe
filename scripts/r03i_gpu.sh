#!/bin/bash
# Round 3: the multi-rank bench rehearsed on one GPU (2 ranks on device 0,
# gloo), then the GPU suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r03i
mkdir -p "$OUT"
step() {
    local name=$1 lim=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -n 1 "$OUT/$name.log" | cut -c1-400
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step rehearsal_n2 300 env MIRT_BENCH_SHARE_GPU=1 python bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu --no-host
step rehearsal_n4 300 env MIRT_BENCH_SHARE_GPU=1 python bench.py --gpus 4 --steps 20 --warmup 5 --no-cpu --no-host
step pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
echo done
