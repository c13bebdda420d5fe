#!/bin/bash
# Round 5, session z: the bounce launch of the timed shape alone under the
# kernel trace (roofline.kernel_ms_trace_check against this round's counter
# pass).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05z
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_exclusive -o run -- python3 bench.py --no-cpu --no-host --pipeline 1 --bounce-blocks 384 --steps 20 --warmup 5 > $OUT/prof_exclusive.log 2>&1 || { tail -5 $OUT/prof_exclusive.log; exit 1; }
python3 scripts/exclusive_trace.py $OUT/prof_exclusive/run_kernel_trace.csv --pmc profiles/r05_pmc_bound_1080p_10k.json
