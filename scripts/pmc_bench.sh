#!/bin/bash
# Counter passes over the bench's OWN command (the timed configuration:
# `pipeline` contexts x `bounce_blocks` workgroups; rocprofv3 --pmc collects
# per dispatch, so it serialises the dispatches it counts -- the counters
# describe each kernel of the timed launch shape, not the overlap itself).
# One small counter set per pass, each under its own kill timeout, within
# 8 SQ / 4 TCC / 4 TCP / 2 TA / 2 TD / 2 GRBM counters. Set 1 carries the
# roofline's numerator, its time and its access shape in ONE pass
# (SQ_INSTS_VMEM_RD, GRBM_GUI_ACTIVE, TCP_TOTAL_CACHE_ACCESSES_sum):
#   scripts/pmc_bench.sh <tag> [bench.py arguments]
# Summarise: scripts/pmc_summary.py gpurun_out/<tag> --pattern 'bench.*' --bounce-grid 98304 --json ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
SETS=(
 "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU GRBM_GUI_ACTIVE TCP_TOTAL_CACHE_ACCESSES_sum"
 "TA_TA_BUSY_sum GRBM_GUI_ACTIVE"
 "TD_TD_BUSY_sum GRBM_GUI_ACTIVE"
 "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"
 "TCP_TCC_READ_REQ_LATENCY_sum GRBM_GUI_ACTIVE"
 "TCC_HIT_sum TCC_MISS_sum"
 "FETCH_SIZE"
 "WRITE_SIZE"
 "SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE"
)
i=0
for cs in "${SETS[@]}"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $cs --output-format csv -d "$OUT/bench.$i" -o run -- \
      python3 bench.py --no-cpu --no-host "$@" > "$OUT/bench.$i.log" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "set $i rc=$rc"; grep -m2 -i "error" "$OUT/bench.$i.log"; exit $rc; fi
done
echo done
