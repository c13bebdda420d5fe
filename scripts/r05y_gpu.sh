#!/bin/bash
# Round 5, session y: the counter passes of the bench's own command on this
# round's kernels (profiles/r05_pmc_bound_1080p_10k.json), then an A/B of the
# lanes' shared accumulation buffer (the ordered fold per fresh frame).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05y
mkdir -p $OUT
timeout -k 10 900 ./scripts/pmc_bench.sh r05y/pmc_1080p_10k --steps 20 > $OUT/pmc_10k.log 2>&1 || { echo "pmc failed"; tail -5 $OUT/pmc_10k.log; exit 1; }
tail -1 $OUT/pmc_10k.log
timeout -k 10 400 python scripts/ab_libs.py ab/libmirt_base.so ab/libmirt_noshare.so --workload 1080p_10k --steps 20 --rounds 3 > $OUT/ab_share.log 2>&1 || { echo "ab failed"; tail -20 $OUT/ab_share.log; exit 1; }
grep BEST $OUT/ab_share.log
