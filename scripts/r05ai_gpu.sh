#!/bin/bash
# Round 5, session ai: the other BASELINE configs on one GPU through the
# round-5 bench (mirt_multi, frames delivered to host memory).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05ai
mkdir -p $OUT
for wl in 1080p_100k 4k_10k 4k_1m_4spp; do
  timeout -k 10 500 python bench.py --no-cpu --no-host --workload $wl > $OUT/bench_$wl.log 2>&1 || { echo "$wl failed"; tail -5 $OUT/bench_$wl.log; exit 1; }
  python3 -c "
import json
t=open('$OUT/bench_$wl.log').read(); d=json.loads(t[t.index('{\"metric'):].split('\n')[0])
rw=d['reference_work']
print('$wl', d['value'], d['ms_per_step'], 'dev', d['device_resident_mrays_s'], 'd1', d['depth1_mrays_s'], 'phases', d['phases_under_overlap_ms'], 'serial', rw['serial_launch']['primary_ms'], rw['serial_launch']['bounce_ms'], 'frac', d['roofline']['frac'], 'ok', d['last_frame_equals_one_context'])"
done
