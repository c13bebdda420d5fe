#!/bin/bash
# Round 4: configs[2] (1080p / 100k) schedule sweep -- refill threshold,
# persistent bounce workgroups, contexts in flight -- two passes each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04h
mkdir -p "$OUT"
B="python3 bench.py --no-cpu --no-host --steps 20 --warmup 5 --workload 1080p_100k"
run() {
    local name=$1; shift
    timeout -k 10 120 $B "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -3 "$OUT/$name.log"; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open('$OUT/$name.log') if l.startswith('{')][-1]); print('$name', d['value'], d['reference_work']['bounce_launch_ms_under_overlap'], d['reference_work']['primary_launch_ms_under_overlap'])"
}
for pass in 1 2; do
  run base_$pass
  for t in 12 16 24 28; do run thr${t}_$pass --opt 5=$t; done
  for bb in 256 512 640; do run bb${bb}_$pass --bounce-blocks $bb; done
  for p in 3 6; do run p${p}_$pass --pipeline $p; done
done
echo done
