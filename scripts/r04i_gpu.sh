#!/bin/bash
# Round 4: counter passes of the bench's own command for the 4K workloads
# (the vmem roofline of every BASELINE config), the multi tests, then a
# configs[2] (1080p / 100k) schedule sweep.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04i
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_multi.py -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_multi.log" 2>&1 || { tail -20 "$OUT/pytest_multi.log"; exit 1; }
tail -1 "$OUT/pytest_multi.log"
timeout -k 10 600 ./scripts/pmc_bench.sh r04i/pmc_4k_10k --steps 20 --workload 4k_10k > "$OUT/pmc_4k_10k.log" 2>&1 || { echo "pmc 4k_10k failed"; tail -5 "$OUT/pmc_4k_10k.log"; exit 1; }
timeout -k 10 900 ./scripts/pmc_bench.sh r04i/pmc_4k_1m_4spp --steps 10 --warmup 2 --workload 4k_1m_4spp > "$OUT/pmc_4k_1m.log" 2>&1 || { echo "pmc 4k_1m failed"; tail -5 "$OUT/pmc_4k_1m.log"; exit 1; }
echo pmc done
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
  run tail2_$pass --tail-grid 2
done
echo done
