#!/bin/bash
# Round 5, session o: the gather probe's access mix (dependent chains, L2
# misses, five waves per SIMD) with its TD / TA busy counter passes -- what
# the bounce kernel's TD-busy-per-instruction says.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05o
mkdir -p "$OUT"
timeout -k 10 120 ./scripts/td_probe --mix > $OUT/mix.json 2> $OUT/mix.err || { cat $OUT/mix.err; exit 1; }
cat $OUT/mix.json
i=0
for cs in "TD_TD_BUSY_sum GRBM_GUI_ACTIVE" "TA_TA_BUSY_sum GRBM_GUI_ACTIVE" "SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE TCP_TOTAL_CACHE_ACCESSES_sum" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $cs --output-format csv -d "$OUT/pmc.$i" -o run -- ./scripts/td_probe --mix > "$OUT/pmc.$i.log" 2>&1 || { echo "pmc set $i failed"; tail -5 "$OUT/pmc.$i.log"; exit 1; }
done
ls -R $OUT | head -30
# kernel-like mixes (VALU and LDS per load as the bounce kernel) at its occupancy
python3 scripts/td_mix_summary.py $OUT > $OUT/summary.txt && cat $OUT/summary.txt
