#!/bin/bash
# Round 4: the frame's HIP events (ev0/ev1 timing + three phase events per
# frame) off in the timed loop -- the bench's N = 1 loop through
# scripts/shard_times.py (4 ctxs, 1 frame per launch, 384 bounce WGs), K = 20
# and K = 100, interleaved rounds; then the N = 8 shard emulation.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04aa
mkdir -p $OUT
for r in 1 2 3; do
  for lib in base noev; do
    for k in 20 100; do
      timeout -k 10 120 env MIRT_LIB=ab/libmirt_$lib.so python3 scripts/shard_times.py --pipeline 4 --batch 1 --worlds 1 --steps $k > $OUT/n1_${lib}_k${k}_r$r.log 2>&1 || { tail -5 $OUT/n1_${lib}_k${k}_r$r.log; exit 1; }
      echo "$lib k$k r$r $(grep '^{' $OUT/n1_${lib}_k${k}_r$r.log | tail -1 | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["min_per_rank_mrays_s"])')"
    done
  done
done
export GPU_MAX_HW_QUEUES=16
for lib in base noev; do
  timeout -k 10 150 env MIRT_LIB=ab/libmirt_$lib.so python3 scripts/shard_times.py --pipeline 8 --steps 5 --copy --batch 4 --worlds 8 --tail-grid 2 > $OUT/emu8_$lib.log 2>&1 || { tail -5 $OUT/emu8_$lib.log; exit 1; }
  echo "emu8 $lib $(grep '^{' $OUT/emu8_$lib.log | tail -1 | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["pred_job_mrays_s_no_gather"])')"
done
