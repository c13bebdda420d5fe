#!/bin/bash
# Round 5, session bm (final confirmation of HEAD, rebuilt library; earlier:
# the N > 1 line saved before the secondary delivery's leg): the whole GPU
# suite (the same-device N = 2 rehearsal runs the new launcher path), the
# smoke test and the driver's bench command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05bm
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
timeout -k 10 400 python bench.py --gpus 2 --same-device --no-cpu --no-host > $OUT/bench_n2_rehearsal.log 2>&1 || { echo "n2 rehearsal failed"; tail -20 $OUT/bench_n2_rehearsal.log; exit 1; }
grep -m1 '"metric"' $OUT/bench_n2_rehearsal.log | cut -c1-160
ls -R $OUT | head -20
