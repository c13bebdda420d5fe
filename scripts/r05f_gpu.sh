#!/bin/bash
# Round 5, session f: the continuation queue (parity, then the blocking
# call with it off / on), the N = 1 loop sweep, the inline-sphere A/B and
# the gather probe's access mix with its counter passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05f
mkdir -p "$OUT"
step() {
    local name=$1 lim=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -n 3 "$OUT/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return $rc
}
step ptr_probe 120 python scripts/ptr_query_probe.py
step pytest_cq 400 python -u -m pytest tests/test_cont_queue.py -m gpu -x -v --timeout 200 --timeout-method thread || exit 1
step cq_ab 400 python scripts/cq_ab.py --rounds 3
grep '"best_ms"' $OUT/cq_ab.log
step n1_sweep 600 python scripts/n1_sweep.py --lanes 4,8 --queues 4,16 --steps 20,100
cat $OUT/n1_sweep.log
step pytest_parity 600 python -u -m pytest tests/test_gpu_parity.py tests/test_full_frames.py tests/test_multi.py -m gpu -x -q --timeout 200 --timeout-method thread || exit 1
step ab_inline 900 python scripts/ab_libs.py ab/libmirt_base.so ab/libmirt_inline.so --rounds 2 --steps 100
grep BEST $OUT/ab_inline.log
bash scripts/r05e_gpu.sh
echo done
