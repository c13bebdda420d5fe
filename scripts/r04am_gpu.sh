#!/bin/bash
# Round 4: frames in flight at N = 1 on the final kernels -- 3 / 4 / 5 / 6
# contexts, and 4 with 320 / 448 bounce workgroups, K = 20, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04am
mkdir -p $OUT
v() { grep '^{' $1 | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"])'; }
for r in 1 2; do
  for a in "--pipeline 4" "--pipeline 3" "--pipeline 5" "--pipeline 6" "--bounce-blocks 320" "--bounce-blocks 448"; do
    n=$(echo $a | tr -d '-' | tr ' ' '_')
    timeout -k 10 120 python3 bench.py --no-cpu --no-host --steps 20 --warmup 5 $a > $OUT/${n}_r$r.log 2>&1 || { tail -5 $OUT/${n}_r$r.log; exit 1; }
    echo "$a r$r $(v $OUT/${n}_r$r.log)"
  done
done
