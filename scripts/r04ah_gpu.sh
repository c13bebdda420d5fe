#!/bin/bash
# Round 4: the blocking call's first bounces queued in tile order (one queue
# atomic per workgroup; frames in flight keep the octant grouping) -- the
# whole GPU suite, the blocking frame, the bench line twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04ah
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 120 python scripts/blocking_frame.py > $OUT/blocking.log 2>&1 || { tail -5 $OUT/blocking.log; exit 1; }
tail -1 $OUT/blocking.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in d if k.endswith("_ms")}, d["frames_equal"])'
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > $OUT/bench_r$r.log 2>&1 || { tail -5 $OUT/bench_r$r.log; exit 1; }
  grep '^{' $OUT/bench_r$r.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["host_blocking_mrays_s"], d["host_blocking_ms"], d["host_blocking_pageable_mrays_s"], d["host_blocking_after_burst"]["pinned_mrays_s"], d["host_inclusive_mrays_s"])'
done
