#!/bin/bash
# Round 4: the burst's end at K = 20 (1080p/10k): kernel traces of the
# driver's command with the last launches on the full bounce grid (--tail-grid)
# and the values of K = 20 runs, rounds interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04m
mkdir -p "$OUT"
for tg in 1 2 4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace_tg$tg" -o run -- python3 bench.py --no-cpu --no-host --steps 20 --warmup 5 --tail-grid $tg > "$OUT/trace_tg$tg.log" 2>&1 || { echo "trace $tg failed"; exit 1; }
done
run() {
    local name=$1; shift
    timeout -k 10 180 python3 bench.py --no-cpu --no-host --steps 20 --warmup 5 "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -3 "$OUT/$name.log"; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open('$OUT/$name.log') if l.startswith('{')][-1]); print('$name', d['value'])"
}
for pass in 1 2 3; do
  for tg in 0 1 2 4; do run tg${tg}_$pass --tail-grid $tg; done
done
echo done
