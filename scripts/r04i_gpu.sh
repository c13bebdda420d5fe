#!/bin/bash
# Round 4: counter passes of the bench's own command for the 4K workloads
# (the vmem roofline of every BASELINE config), then the multi tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04i
mkdir -p "$OUT"
timeout -k 10 600 ./scripts/pmc_bench.sh r04i/pmc_4k_10k --steps 20 --workload 4k_10k > "$OUT/pmc_4k_10k.log" 2>&1 || { echo "pmc 4k_10k failed"; tail -5 "$OUT/pmc_4k_10k.log"; exit 1; }
timeout -k 10 900 ./scripts/pmc_bench.sh r04i/pmc_4k_1m_4spp --steps 10 --warmup 2 --workload 4k_1m_4spp > "$OUT/pmc_4k_1m.log" 2>&1 || { echo "pmc 4k_1m failed"; tail -5 "$OUT/pmc_4k_1m.log"; exit 1; }
echo pmc done
timeout -k 10 300 python -u -m pytest tests/test_multi.py -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/pytest_multi.log" 2>&1; tail -3 "$OUT/pytest_multi.log"
