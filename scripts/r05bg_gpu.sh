#!/bin/bash
# Round 5, session bg (the round's final record, final library): the whole GPU suite, the smoke
# test, the driver's bench command (CPU baseline and blocking leg included),
# and the kernel trace of the same timed loop (rocprofv3 --kernel-trace
# --stats) for profiles/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05bg
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -10 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 420 python bench.py > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -20 $OUT/bench.log; exit 1; }
python3 -c "
import json
t=open('$OUT/bench.log').read(); d=json.loads(t[t.index('{\"metric'):].split('\n')[0])
print('value', d['value'], 'ms', d['ms_per_step'], 'dev', d['device_resident_mrays_s'], 'd1', d['depth1_mrays_s'], 'blocking', d.get('host_blocking_mrays_s'), 'frac', d['roofline']['frac'], 'cpu', d.get('cpu_baseline',{}).get('value'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_timed -o run -- python3 bench.py --no-cpu --no-host > $OUT/prof_timed.log 2>&1 || { echo "trace failed"; tail -10 $OUT/prof_timed.log; exit 1; }
grep -m1 '"metric"' $OUT/prof_timed.log | cut -c1-200
ls -R $OUT | head -20
