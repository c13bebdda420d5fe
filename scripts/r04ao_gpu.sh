#!/bin/bash
# Round 4: bench.py's N = 1 default of 8 hardware queues against the box's 4
# (--hw-queues 0), K = 20 and K = 100, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04ao
mkdir -p $OUT
v() { grep '^{' $1 | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["config"]["hw_queues"])'; }
for r in 1 2 3; do
  for q in -1 0; do
    timeout -k 10 120 python3 bench.py --no-cpu --no-host --steps 20 --warmup 5 --hw-queues $q > $OUT/k20_q${q}_r$r.log 2>&1 || { tail -5 $OUT/k20_q${q}_r$r.log; exit 1; }
    echo "K20 hw-queues=$q r$r $(v $OUT/k20_q${q}_r$r.log)"
  done
done
for q in -1 0; do
  timeout -k 10 120 python3 bench.py --no-cpu --no-host --steps 100 --warmup 5 --hw-queues $q > $OUT/k100_q$q.log 2>&1 || { tail -5 $OUT/k100_q$q.log; exit 1; }
  echo "K100 hw-queues=$q $(v $OUT/k100_q$q.log)"
  timeout -k 10 120 python3 bench.py --no-cpu --no-host --steps 20 --warmup 5 --workload 1080p_100k --hw-queues $q > $OUT/k20_100k_q$q.log 2>&1 || { tail -5 $OUT/k20_100k_q$q.log; exit 1; }
  echo "100k hw-queues=$q $(v $OUT/k20_100k_q$q.log)"
done
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $OUT/bench_full.log 2>&1 || { tail -5 $OUT/bench_full.log; exit 1; }
grep '^{' $OUT/bench_full.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("full", d["value"], d["host_inclusive_mrays_s"], d["host_blocking_mrays_s"], d["config"]["hw_queues"])'
