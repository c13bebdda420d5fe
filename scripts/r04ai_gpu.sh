#!/bin/bash
# Round 4: MIRT_OPT_QUEUE_ORDER -- its parity test, then tile order vs octant
# groups for frames in flight: the N = 8 per-shard emulation and the N = 1
# timed loop (10k, 100k), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04ai
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "queue_orders or bounce_modes" --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2; do
  for o in 1 2; do
    timeout -k 10 120 python3 bench.py --no-cpu --no-host --steps 20 --warmup 5 --opt 18=$o > $OUT/bench_o${o}_r$r.log 2>&1 || { tail -5 $OUT/bench_o${o}_r$r.log; exit 1; }
    echo "10k order=$o r$r $(grep '^{' $OUT/bench_o${o}_r$r.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')"
    timeout -k 10 120 python3 bench.py --no-cpu --no-host --steps 20 --warmup 5 --workload 1080p_100k --opt 18=$o > $OUT/bench100k_o${o}_r$r.log 2>&1 || { tail -5 $OUT/bench100k_o${o}_r$r.log; exit 1; }
    echo "100k order=$o r$r $(grep '^{' $OUT/bench100k_o${o}_r$r.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])')"
  done
done
export GPU_MAX_HW_QUEUES=16
for r in 1 2; do
  for o in 1 2; do
    timeout -k 10 150 python3 scripts/shard_times.py --pipeline 8 --steps 5 --copy --batch 4 --worlds 8 --tail-grid 2 --opt 18=$o > $OUT/emu8_o${o}_r$r.log 2>&1 || { tail -5 $OUT/emu8_o${o}_r$r.log; exit 1; }
    echo "emu8 order=$o r$r $(grep '^{' $OUT/emu8_o${o}_r$r.log | tail -1 | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["pred_job_mrays_s_no_gather"])')"
  done
done
