#!/bin/bash
# Round 3: camera packets touch their inner children's PNodes (scalar cache)
# before the step's tests (MIRT_PACKET_PREFETCH): parity, then A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r03q
mkdir -p "$OUT"
step() {
    local name=$1 lim=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -n 4 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
for wl in 1080p_10k 1080p_100k 4k_1m_4spp; do
    step ab_$wl 600 python scripts/ab_libs.py ab/libmirt_pf0.so ab/libmirt_pf1.so --workload $wl --steps 20 --rounds 2
done
echo done
