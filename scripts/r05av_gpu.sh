#!/bin/bash
# Round 5, session av: the frame D2H as a 2D copy (MIRT_D2H_2D) instead of 1D (no blit
# kernel on the compute queue) against the default kind, N = 1 loop into host
# memory; golden check of the variant, three interleaved rounds, then the
# kernel trace of the variant's loop.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05av
mkdir -p $OUT
for r in 1 2 3; do
  for v in base d2h2d; do
    MIRT_LIB=$PWD/ab/libmirt_$v.so timeout -k 10 300 python bench.py --no-cpu --no-host > $OUT/bench_${v}_r$r.log 2>&1 || { echo "bench $v failed"; tail -8 $OUT/bench_${v}_r$r.log; exit 1; }
    python3 -c "
import json
t=open('$OUT/bench_${v}_r$r.log').read(); d=json.loads(t[t.index('{\"metric'):].split('\n')[0])
print('$v r$r', d['value'], d['ms_per_step'], 'dev', d['device_resident_mrays_s'], 'd1', d['depth1_mrays_s'], 'ok', d['last_frame_equals_one_context'])"
  done
done
MIRT_LIB=$PWD/ab/libmirt_d2h2d.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_d2h2d -o run -- python3 bench.py --no-cpu --no-host > $OUT/prof_d2h2d.log 2>&1 || { echo "trace failed"; tail -5 $OUT/prof_d2h2d.log; exit 1; }
grep -c rocclr_copyBuffer $OUT/prof_d2h2d/run_kernel_trace.csv || true
