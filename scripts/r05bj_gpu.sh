#!/bin/bash
# Round 5, session bj (the final tree): the driver's bench command (with the
# in-process blocking leg after the burst now in the line), the other BASELINE
# configs through the same bench, and the N = 1/2/4/8 per-shard emulation of
# the mirt_multi schedule (host-direct, the headline's delivery).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05bj
mkdir -p $OUT
timeout -k 10 420 python bench.py > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench.log; exit 1; }
python3 -c "
import json
t=open('$OUT/bench.log').read(); d=json.loads(t[t.index('{\"metric'):].split('\n')[0])
print('value', d['value'], 'ms', d['ms_per_step'], 'dev', d['device_resident_mrays_s'], 'blocking', d.get('host_blocking_mrays_s'), 'after_burst', d.get('host_blocking_after_burst'))"
for w in 1080p_100k 4k_10k 4k_1m_4spp; do
  timeout -k 10 400 python bench.py --workload $w --no-cpu --no-host > $OUT/bench_$w.log 2>&1 || { echo "bench $w failed"; tail -20 $OUT/bench_$w.log; exit 1; }
  python3 -c "
import json
t=open('$OUT/bench_$w.log').read(); d=json.loads(t[t.index('{\"metric'):].split('\n')[0])
print('$w', d['value'], 'ms', d['ms_per_step'], 'dev', d['device_resident_mrays_s'], 'same', d['last_frame_equals_one_context'])"
done
timeout -k 10 600 python scripts/multi_emulate.py --worlds 1,2,4,8 --delivery host-direct > $OUT/emu_direct.log 2>&1 || { echo "emulation failed"; tail -20 $OUT/emu_direct.log; exit 1; }
tail -12 $OUT/emu_direct.log
