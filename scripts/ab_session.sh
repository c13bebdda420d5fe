#!/bin/bash
# One GPU session of a kernel A/B: the full GPU suite on the in-tree library
# (the candidate), then scripts/ab_libs.py on the libraries for the headline
# and the deep-tree workloads, two interleaved rounds each.
#   bash scripts/ab_session.sh NAME ab/libmirt_a.so ab/libmirt_b.so [more.so ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
NAME=$1
shift
OUT=gpurun_out/$NAME
mkdir -p "$OUT"
step() {
    local name=$1 lim=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -n 2 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
for wl in 1080p_10k 1080p_100k 4k_1m_4spp; do
    step ab_$wl 600 python scripts/ab_libs.py "$@" --workload $wl --steps 20 --rounds 2
done
echo done
