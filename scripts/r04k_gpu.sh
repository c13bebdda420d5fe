#!/bin/bash
# Round 4: persistent bounce workgroups per launch with four frames in flight
# (bench --bounce-blocks; 384 = 1.5 per CU since round 2), rounds interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04k
mkdir -p "$OUT"
run() {
    local name=$1; shift
    timeout -k 10 180 python3 bench.py --no-cpu --no-host --steps 20 --warmup 5 "$@" > "$OUT/$name.log" 2>&1 || { echo "$name failed"; tail -3 "$OUT/$name.log"; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open('$OUT/$name.log') if l.startswith('{')][-1]); print('$name', d['value'], d['reference_work']['bounce_launch_ms_under_overlap'], d['reference_work']['primary_launch_ms_under_overlap'])"
}
for pass in 1 2 3; do
  for bb in 384 448 512 576; do run 10k_bb${bb}_$pass --bounce-blocks $bb; done
done
for pass in 1 2; do
  for bb in 384 512; do run 4k_bb${bb}_$pass --bounce-blocks $bb --workload 4k_10k; done
  for bb in 384 512; do run 4k1m_bb${bb}_$pass --bounce-blocks $bb --workload 4k_1m_4spp; done
  for bb in 384 512; do run 100k_bb${bb}_$pass --bounce-blocks $bb --workload 1080p_100k; done
done
echo done
