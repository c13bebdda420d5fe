#!/bin/bash
# Round 4: counter passes of the bench's own command (1080p/10k and 100k) for
# the vmem roofline, then the bench itself and its kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04b
mkdir -p "$OUT"
timeout -k 10 600 ./scripts/pmc_bench.sh r04b/pmc_1080p_10k --steps 20 > "$OUT/pmc_10k.log" 2>&1 || { echo "pmc 10k failed"; tail -5 "$OUT/pmc_10k.log"; exit 1; }
timeout -k 10 600 ./scripts/pmc_bench.sh r04b/pmc_1080p_100k --steps 20 --workload 1080p_100k > "$OUT/pmc_100k.log" 2>&1 || { echo "pmc 100k failed"; tail -5 "$OUT/pmc_100k.log"; exit 1; }
echo pmc done
