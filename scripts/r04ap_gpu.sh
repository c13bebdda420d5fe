#!/bin/bash
# Round 4, last commit: GPU suite, smoke and the driver's bench command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04ap
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || { tail -5 $OUT/bench.log; exit 1; }
grep '^{' $OUT/bench.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["host_inclusive_mrays_s"], d["host_blocking_mrays_s"], d["roofline"]["frac"], d["cpu_baseline"]["value"])'
