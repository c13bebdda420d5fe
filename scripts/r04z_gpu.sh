#!/bin/bash
# Round 4 (final tree): counter passes of the 4K workloads' bounce kernel and
# the one-frame split at N = 8 emulated per shard (the bench's N > 1
# defaults: 8 ctxs, 4 frames per launch, copy stream, 16 queues, tail grid 2).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04z
mkdir -p "$OUT"
timeout -k 10 600 ./scripts/pmc_bench.sh r04z/pmc_4k_10k --steps 20 --workload 4k_10k > "$OUT/pmc_4k_10k.log" 2>&1 || { echo "pmc 4k_10k failed"; tail -5 "$OUT/pmc_4k_10k.log"; exit 1; }
timeout -k 10 900 ./scripts/pmc_bench.sh r04z/pmc_4k_1m_4spp --steps 10 --warmup 2 --workload 4k_1m_4spp > "$OUT/pmc_4k_1m.log" 2>&1 || { echo "pmc 4k_1m failed"; tail -5 "$OUT/pmc_4k_1m.log"; exit 1; }
export GPU_MAX_HW_QUEUES=16
for r in 1 2; do
  timeout -k 10 150 python3 scripts/shard_times.py --pipeline 8 --steps 5 --copy --batch 4 --worlds 1,8 --tail-grid 2 > "$OUT/emu8_r$r.log" 2>&1 || { echo "emu failed"; tail -5 "$OUT/emu8_r$r.log"; exit 1; }
  grep '^{' "$OUT/emu8_r$r.log" | cut -c1-300
done
echo done
