#!/bin/bash
# Round 3, final tree: PMC passes of the bench's own command for every
# BASELINE workload (scripts/pmc_bench.sh; summaries by scripts/pmc_summary.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
timeout -k 10 280 bash scripts/pmc_bench.sh r03zc/pmc_1080p_10k --steps 20 --warmup 5 &&
timeout -k 10 280 bash scripts/pmc_bench.sh r03zc/pmc_1080p_100k --workload 1080p_100k --steps 20 --warmup 5 &&
timeout -k 10 280 bash scripts/pmc_bench.sh r03zc/pmc_4k_10k --workload 4k_10k --steps 20 --warmup 5 &&
timeout -k 10 330 bash scripts/pmc_bench.sh r03zc/pmc_4k_1m_4spp --workload 4k_1m_4spp --steps 20 --warmup 5
