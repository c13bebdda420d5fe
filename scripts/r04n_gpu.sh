#!/bin/bash
# Round 4: frames in flight written in place into page-locked memory
# (MIRT_OPT_ZERO_COPY 2) vs a DMA behind each frame (1): bench host leg.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04n
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "shared_accumulation or registered or private" > "$OUT/pytest.log" 2>&1 || { tail -20 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
run() {
    local name=$1; shift
    timeout -k 10 180 python3 bench.py --no-cpu --steps 20 --warmup 5 "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -3 "$OUT/$name.log"; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open('$OUT/$name.log') if l.startswith('{')][-1]); print('$name', d['value'], d['host_inclusive_mrays_s'], d['host_blocking_mrays_s'], d['host_blocking_registered_mrays_s'], d['host_blocking_pageable_mrays_s'])"
}
for pass in 1 2 3; do
  run zc1_$pass
  run zc2_$pass --opt 17=2
done
echo done
