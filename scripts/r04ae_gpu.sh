#!/bin/bash
# Round 4: the chain handoff from SPARSE waves only (quad drain, solo) --
# its parity tests, then the lone frame (blocking call), the pipelined bench
# loop and the N = 8 per-shard emulation with it on and off.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04ae
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_chains.py tests/test_gpu_parity.py -k "chains or bounce_modes or golden" -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_chains.log 2>&1 || { tail -30 $OUT/pytest_chains.log; exit 1; }
tail -1 $OUT/pytest_chains.log
for o in 0 1; do
  timeout -k 10 120 python scripts/blocking_frame.py --opt 18=$o > $OUT/blocking_c$o.log 2>&1 || { tail -5 $OUT/blocking_c$o.log; exit 1; }
  echo "chains=$o $(tail -1 $OUT/blocking_c$o.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ("pinned_ms","pageable_ms","kernels_ms","frames_equal")})')"
done
for r in 1 2; do
  for o in 0 1; do
    timeout -k 10 120 python3 bench.py --no-cpu --no-host --steps 20 --warmup 5 --opt 18=$o > $OUT/bench_c${o}_r$r.log 2>&1 || { tail -5 $OUT/bench_c${o}_r$r.log; exit 1; }
    echo "bench chains=$o r$r $(grep '^{' $OUT/bench_c${o}_r$r.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["reference_work"]["serial_launch"]["frame_ms"])')"
    timeout -k 10 120 python3 bench.py --no-cpu --no-host --steps 20 --warmup 5 --workload 1080p_100k --opt 18=$o > $OUT/bench100k_c${o}_r$r.log 2>&1 || { tail -5 $OUT/bench100k_c${o}_r$r.log; exit 1; }
    echo "bench100k chains=$o r$r $(grep '^{' $OUT/bench100k_c${o}_r$r.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["reference_work"]["serial_launch"]["frame_ms"])')"
  done
done
export GPU_MAX_HW_QUEUES=16
for o in 0 1; do
  timeout -k 10 150 python3 scripts/shard_times.py --pipeline 8 --steps 5 --copy --batch 4 --worlds 8 --tail-grid 2 --opt 18=$o > $OUT/emu8_c$o.log 2>&1 || { tail -5 $OUT/emu8_c$o.log; exit 1; }
  echo "emu8 chains=$o $(grep '^{' $OUT/emu8_c$o.log | tail -1 | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["pred_job_mrays_s_no_gather"])')"
done
