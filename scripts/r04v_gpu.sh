#!/bin/bash
# Round 4: the blocking frame's zero-copy stores -- mirt_host_alloc memory
# non-coherent / write-combined, and non-temporal pixel stores, against the
# build as committed.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04v
mkdir -p $OUT
for lib in base nc wc nt base; do
  timeout -k 10 120 env MIRT_LIB=ab/libmirt_$lib.so python scripts/blocking_frame.py > $OUT/blocking_$lib.log 2>&1 || { tail -5 $OUT/blocking_$lib.log; exit 1; }
  echo "$lib $(tail -1 $OUT/blocking_$lib.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in d if k.endswith("_ms")}, d["frames_equal"])')"
done
