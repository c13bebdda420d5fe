#!/bin/bash
# Round 4 (final tree): GPU parity suite, smoke, the driver's
# bench command (K = 20), K = 100, the other workloads, the rocprofv3 kernel
# trace of the driver's command, the blocking frame by destination.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04al
mkdir -p "$OUT"
step() {
    local name=$1 lim=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -n 1 "$OUT/$name.log" | cut -c1-200
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --steps 20 --warmup 5
step bench_k100 300 python bench.py --no-cpu --no-host --steps 100 --warmup 5
step prof_timed 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_timed" -o run -- python3 bench.py --no-cpu --no-host --steps 20 --warmup 5
for wl in 1080p_100k 4k_10k 4k_1m_4spp; do
  step bench_$wl 600 python bench.py --no-cpu --no-host --steps 20 --warmup 5 --workload $wl
done
step blocking 120 python scripts/blocking_frame.py
step rehearsal_n4 300 env MIRT_BENCH_SHARE_GPU=1 python bench.py --gpus 4 --steps 20 --warmup 5 --no-cpu --no-host
echo done
