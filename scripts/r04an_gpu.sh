#!/bin/bash
# Round 4: frames in flight at N = 1 with 8 hardware queues (GPU_MAX_HW_QUEUES
# raised before the runtime starts) -- 4 / 5 / 6 / 8 contexts, K = 20, against
# the box's 4 queues with 4 contexts.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04an
mkdir -p $OUT
v() { grep '^{' $1 | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["config"]["hw_queues"])'; }
for r in 1 2; do
  timeout -k 10 120 python3 bench.py --no-cpu --no-host --steps 20 --warmup 5 > $OUT/q4_p4_r$r.log 2>&1 || { tail -5 $OUT/q4_p4_r$r.log; exit 1; }
  echo "q4 p4 r$r $(v $OUT/q4_p4_r$r.log)"
  for p in 4 5 6 8; do
    timeout -k 10 120 env GPU_MAX_HW_QUEUES=8 python3 bench.py --no-cpu --no-host --steps 20 --warmup 5 --pipeline $p > $OUT/q8_p${p}_r$r.log 2>&1 || { tail -5 $OUT/q8_p${p}_r$r.log; exit 1; }
    echo "q8 p$p r$r $(v $OUT/q8_p${p}_r$r.log)"
  done
done
