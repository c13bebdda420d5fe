#!/bin/bash
# Round 3, second GPU session: the GPU parity suite (shared accumulation
# across frames in flight, full-frame goldens of BASELINE configs[2]-[4],
# drop-in rebinding, orphan phantom leaves), the new bench line, the
# one-frame split emulated with batched frames / more hardware queues, and
# the PMC passes of the bench's own command. Each GPU step has its own time
# limit; a fault / abort / timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r03b
mkdir -p "$OUT"
step() {
    local name=$1 lim=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -n 3 "$OUT/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --steps 20 --warmup 5
for b in 1 2 4; do
    step strong_batch$b 300 python3 scripts/shard_times.py --pipeline 4 --batch $b --steps 60
done
step strong_q8_p8 300 env GPU_MAX_HW_QUEUES=8 python3 scripts/shard_times.py --pipeline 8 --steps 80
step strong_q8_p6 300 env GPU_MAX_HW_QUEUES=8 python3 scripts/shard_times.py --pipeline 6 --steps 60
step pmc 1500 bash scripts/pmc_bench.sh r03b/pmc_1080p_10k --steps 20 --warmup 5
echo done
