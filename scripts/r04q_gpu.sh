#!/bin/bash
# Round 4: the blocking frame by destination across the process's phases
# (plain / after torch's context / after bench.py's pipelined leg), then the
# counter passes and the exclusive kernel trace of the final bounce kernel
# (solo drain) at 1080p / 10k and 1080p / 100k.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04q
mkdir -p "$OUT"
timeout -k 10 180 python scripts/blocking_frame.py --phases plain,torch,burst > "$OUT/blocking_phases.log" 2>&1 || { tail -5 "$OUT/blocking_phases.log"; exit 1; }
tail -1 "$OUT/blocking_phases.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_exclusive" -o run -- python3 bench.py --no-cpu --no-host --pipeline 1 --bounce-blocks 384 --steps 20 --warmup 5 > "$OUT/prof_exclusive.log" 2>&1 || { tail -5 "$OUT/prof_exclusive.log"; exit 1; }
timeout -k 10 600 ./scripts/pmc_bench.sh r04q/pmc_1080p_10k --steps 20 > "$OUT/pmc_10k.log" 2>&1 || { echo "pmc 10k failed"; tail -5 "$OUT/pmc_10k.log"; exit 1; }
timeout -k 10 600 ./scripts/pmc_bench.sh r04q/pmc_1080p_100k --steps 20 --workload 1080p_100k > "$OUT/pmc_100k.log" 2>&1 || { echo "pmc 100k failed"; tail -5 "$OUT/pmc_100k.log"; exit 1; }
echo done
