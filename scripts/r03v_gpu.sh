#!/bin/bash
# Round 3: PMC passes of the bench's own command for the headline and for
# 4K/1M (whose bounce kernel is now WALK 4 with batched leaf gates).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
timeout -k 10 900 bash scripts/pmc_bench.sh r03v/pmc_4k_1m_4spp --workload 4k_1m_4spp --steps 20 --warmup 5 &&
timeout -k 10 900 bash scripts/pmc_bench.sh r03v/pmc_1080p_10k --steps 20 --warmup 5
