#!/bin/bash
# Round 5, session d: the N = 1 sweep (lanes / queues / delivery / steps),
# then the A/B of inline-sphere PNode leaf slots (camera packets).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05d
mkdir -p "$OUT"
timeout -k 10 600 python scripts/n1_sweep.py --lanes 4,8 --queues 4,16 --steps 20,100 > $OUT/n1_sweep.log 2>&1 || { cat $OUT/n1_sweep.log; exit 1; }
cat $OUT/n1_sweep.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_full_frames.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_parity.log 2>&1 || { tail -20 $OUT/pytest_parity.log; exit 1; }
tail -1 $OUT/pytest_parity.log
timeout -k 10 900 python scripts/ab_libs.py ab/libmirt_base.so ab/libmirt_inline.so --rounds 3 --steps 100 > $OUT/ab_inline.log 2>&1; rc=$?
grep -v "^{" $OUT/ab_inline.log | tail -4; grep '^{' $OUT/ab_inline.log | python3 -c 'import json,sys
for l in sys.stdin: d=json.loads(l); print(d["lib"][-20:], d["value"], d["device_resident"], d["primary_ms"], d["bounce_ms"], d["serial_primary_ms"], d["depth1"])'
exit $rc
