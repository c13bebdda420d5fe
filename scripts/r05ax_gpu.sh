#!/bin/bash
# Round 5, session ax: MIRT_LAZY_FOLD -- the accumulation / multi / C-loop
# parity tests, then the whole GPU suite, then the bench loop (depth 5 and
# depth 1 in the line) against the build without it, two interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05ax
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_multi.py tests/test_c_dropin.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_acc.log 2>&1 || { echo "acc tests failed"; tail -30 $OUT/pytest_acc.log; exit 1; }
tail -1 $OUT/pytest_acc.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "gpu suite failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for r in 1 2; do
  for v in eager lazy; do
    MIRT_LIB=$PWD/ab/libmirt_$v.so timeout -k 10 300 python bench.py --no-cpu --no-host > $OUT/bench_${v}_r$r.log 2>&1 || { echo "bench $v failed"; tail -8 $OUT/bench_${v}_r$r.log; exit 1; }
    python3 -c "
import json
t=open('$OUT/bench_${v}_r$r.log').read(); d=json.loads(t[t.index('{\"metric'):].split('\n')[0])
print('$v r$r', d['value'], d['ms_per_step'], 'dev', d['device_resident_mrays_s'], 'd1', d['depth1_mrays_s'], 'ok', d['last_frame_equals_one_context'])"
  done
done
