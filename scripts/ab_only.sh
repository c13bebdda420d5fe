#!/bin/bash
# scripts/ab_libs.py on the given libraries at the headline, deep-tree and
# 4K/1M workloads (two interleaved rounds each), no test suite:
#   bash scripts/ab_only.sh NAME ab/libmirt_a.so ab/libmirt_b.so [more.so ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
NAME=$1
shift
OUT=gpurun_out/$NAME
mkdir -p "$OUT"
for wl in 1080p_10k 1080p_100k 4k_1m_4spp; do
    echo "== ab_$wl ($(date +%T))"
    timeout -k 10 600 python scripts/ab_libs.py "$@" --workload $wl --steps 20 --rounds 2 > "$OUT/ab_$wl.log" 2>&1
    rc=$?
    grep BEST "$OUT/ab_$wl.log"
    if [ $rc -ne 0 ]; then echo "stopping after ab_$wl (rc=$rc)"; exit $rc; fi
done
echo done
