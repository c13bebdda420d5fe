#!/bin/bash
# Round 5, session ag: bounce queue segments taken from their end
# (MIRT_QUEUE_REVERSE: the dense tiles' first bounces, appended last, start
# first). Golden check, then interleaved bench rounds with the blocking leg,
# the per-wave drain statistics, and the deep-tree config.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05ag
mkdir -p $OUT
timeout -k 10 200 python scripts/ab_libs.py ab/libmirt_base.so ab/libmirt_rev.so --rounds 0 > $OUT/golden.log 2>&1 || { echo "golden failed"; tail -5 $OUT/golden.log; exit 1; }
grep golden $OUT/golden.log
for r in 1 2 3; do
  for v in base rev; do
    MIRT_LIB=$PWD/ab/libmirt_$v.so timeout -k 10 300 python bench.py --no-cpu > $OUT/bench_${v}_r$r.log 2>&1 || { echo "bench $v failed"; tail -5 $OUT/bench_${v}_r$r.log; exit 1; }
    python3 -c "
import json
t=open('$OUT/bench_${v}_r$r.log').read(); d=json.loads(t[t.index('{\"metric'):].split('\n')[0])
print('$v r$r', d['value'], d['device_resident_mrays_s'], 'blocking_ms', d.get('host_blocking_ms'), 'serial bounce', d['reference_work']['serial_launch']['bounce_ms'], 'ok', d['last_frame_equals_one_context'], d.get('host_blocking_equals_frames'))"
  done
done
for v in base rev; do
  MIRT_LIB=$PWD/ab/libmirt_$v.so timeout -k 10 200 python scripts/bounce_stats.py --shards 1,8 > $OUT/bstats_$v.log 2>&1 || { echo "bstats $v failed"; tail -5 $OUT/bstats_$v.log; exit 1; }
  grep shards $OUT/bstats_$v.log | python3 -c "
import sys,json
for l in sys.stdin: d=json.loads(l); print('$v', 'shards', d['shards'], 'span', d['span_us'], 'dry', d['queue_dry_us_median'], 'end p50/p90', d['wave_end_us_p50'], d['wave_end_us_p90'])"
done
for v in base rev; do
  MIRT_LIB=$PWD/ab/libmirt_$v.so timeout -k 10 300 python bench.py --no-cpu --no-host --workload 1080p_100k > $OUT/bench100k_$v.log 2>&1 || { echo "100k $v failed"; exit 1; }
  python3 -c "
import json
t=open('$OUT/bench100k_$v.log').read(); d=json.loads(t[t.index('{\"metric'):].split('\n')[0])
print('100k $v', d['value'], d['device_resident_mrays_s'], d['last_frame_equals_one_context'])"
done
