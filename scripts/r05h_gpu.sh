#!/bin/bash
# Round 5, session h: continuation-queue diagnostics (lane / quad pushes),
# and the N = 8 schedule sweep in the per-shard emulation (host-direct).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05h
mkdir -p "$OUT"
step() {
    local name=$1 lim=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -n 2 "$OUT/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return $rc
}
step cq_lane 300 python scripts/cq_ab.py --rounds 1 --spheres 10000
cat $OUT/cq_lane.log
MIRT_LIB=$PWD/ab/libmirt_cq_quad.so step cq_quad 300 python scripts/cq_ab.py --rounds 1 --spheres 10000
cat $OUT/cq_quad.log
step sweep8 900 python scripts/multi_emulate.py --worlds 8 --delivery host-direct --sweep 8:4:2,8:2:2,8:1:2,8:3:2,8:5:2,8:4:0,8:4:1,8:4:3,4:4:2,6:4:2,12:4:2,12:2:2,16:2:2,8:2:4
grep -h pred_job $OUT/sweep8.log | python3 -c 'import json,sys
for l in sys.stdin: d=json.loads(l); print(d["lanes"], d["frames_per_launch"], d["tail_grid"], d["pred_job_mrays_s"], max(d["rank_ms_per_frame"]))'
echo done
