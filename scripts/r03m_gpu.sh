#!/bin/bash
# Round 3: the eight-wide quantised bounce walk (MIRT_OPT_BOUNCE_WALK 8):
# its parity tests, then bench A/B against the four-wide walk per workload.
# (The variant lost and was removed after this run: commit 1cb0f72 holds it;
# results in profiles/r03m_walk8_ab/ and DESIGN.md §8.)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r03m
mkdir -p "$OUT"
step() {
    local name=$1 lim=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -n 3 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step pytest_walk8 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -k "walk8 or bounce_modes or pruning" --timeout 300 --timeout-method thread
for wl in 1080p_10k 1080p_100k 4k_1m_4spp; do
    step bench_${wl}_w4 300 python bench.py --steps 20 --warmup 5 --no-cpu --no-host --workload $wl
    step bench_${wl}_w8 300 python bench.py --steps 20 --warmup 5 --no-cpu --no-host --workload $wl --opt 12=8
done
echo done
