#!/bin/bash
# Round 3: A/B of the primary workgroup's octant grouping of first bounces
# (ab/libmirt_group.so vs ab/libmirt_base.so), golden-checked, at 10k / 100k
# / 4K-1M; then the PMC passes of the other workloads' bench commands.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r03e
mkdir -p "$OUT"
step() {
    local name=$1 lim=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; grep BEST "$OUT/$name.log" || tail -n 2 "$OUT/$name.log" | cut -c1-300
    if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step ab_10k 400 python scripts/ab_libs.py ab/libmirt_base.so ab/libmirt_group.so --rounds 3
step ab_100k 400 python scripts/ab_libs.py ab/libmirt_base.so ab/libmirt_group.so --rounds 2 --workload 1080p_100k
step ab_4k1m 600 python scripts/ab_libs.py ab/libmirt_base.so ab/libmirt_group.so --rounds 2 --workload 4k_1m_4spp --steps 20
for wl in 1080p_100k 4k_10k 4k_1m_4spp; do
  step pmc_$wl 1500 bash scripts/pmc_bench.sh r03e/pmc_$wl --steps 20 --warmup 5 --workload $wl
done
echo done
