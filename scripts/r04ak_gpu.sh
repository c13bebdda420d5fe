#!/bin/bash
# Round 4: camera-packet passes chained across the frames-in-flight contexts
# (MIRT_OPT_PRIMARY_CHAIN 19) -- the timed loop K = 20 / 100 at 10k, 100k,
# and the N = 8 per-shard emulation, interleaved with the default.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04ak
mkdir -p $OUT
v() { grep '^{' $1 | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d.get("value", d.get("pred_job_mrays_s_no_gather")))'; }
for r in 1 2 3; do
  for o in 0 1; do
    timeout -k 10 120 python3 bench.py --no-cpu --no-host --steps 20 --warmup 5 --opt 19=$o > $OUT/k20_o${o}_r$r.log 2>&1 || { tail -5 $OUT/k20_o${o}_r$r.log; exit 1; }
    echo "10k K20 chain=$o r$r $(v $OUT/k20_o${o}_r$r.log)"
  done
done
for o in 0 1; do
  timeout -k 10 120 python3 bench.py --no-cpu --no-host --steps 100 --warmup 5 --opt 19=$o > $OUT/k100_o$o.log 2>&1 || { tail -5 $OUT/k100_o$o.log; exit 1; }
  echo "10k K100 chain=$o $(v $OUT/k100_o$o.log)"
  timeout -k 10 120 python3 bench.py --no-cpu --no-host --steps 20 --warmup 5 --workload 1080p_100k --opt 19=$o > $OUT/k20_100k_o$o.log 2>&1 || { tail -5 $OUT/k20_100k_o$o.log; exit 1; }
  echo "100k K20 chain=$o $(v $OUT/k20_100k_o$o.log)"
done
export GPU_MAX_HW_QUEUES=16
for o in 0 1; do
  timeout -k 10 150 python3 scripts/shard_times.py --pipeline 8 --steps 5 --copy --batch 4 --worlds 8 --tail-grid 2 --opt 19=$o > $OUT/emu8_o$o.log 2>&1 || { tail -5 $OUT/emu8_o$o.log; exit 1; }
  echo "emu8 chain=$o $(v $OUT/emu8_o$o.log)"
done
