#!/bin/bash
# Counter probe of the frame kernels, one small counter set per rocprofv3 pass
# (a set beyond the hardware's per-block limits hangs the profiler, so every
# pass runs under its own kill timeout and stays within 8 SQ / 4 TCC / 4 TCP /
# 2 TA / 2 TD / 2 GRBM counters):
#   scripts/pmc_probe.sh <tag> "<trav> <fast> <depth>" ...
# PROBE_ARGS (environment): more scripts/profile_kernel.py arguments, e.g.
#   PROBE_ARGS="--scene bench1000000 --W 3840 --H 2160"
# Summarise with scripts/pmc_summary.py gpurun_out/<tag> [--json out.json].
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
SETS=(
 "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU"
 "TA_TA_BUSY_sum GRBM_GUI_ACTIVE"
 "TD_TD_BUSY_sum GRBM_GUI_ACTIVE"
 "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"
 "TCP_TCC_READ_REQ_LATENCY_sum GRBM_GUI_ACTIVE"
 "TCC_HIT_sum TCC_MISS_sum"
 "FETCH_SIZE"
 "WRITE_SIZE"
 "SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE"
)
for cfg in "$@"; do
  set -- $cfg
  tag=t$1_f$2_d$3
  i=0
  for cs in "${SETS[@]}"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $cs --output-format csv -d "$OUT/$tag.$i" -o run -- \
        python3 scripts/profile_kernel.py --trav $1 --fast $2 --depth $3 --frames 3 ${PROBE_ARGS:-} > "$OUT/$tag.$i.log" 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "$tag set $i rc=$rc"; grep -m2 -i "error" "$OUT/$tag.$i.log"; [ $rc -gt 1 ] && exit $rc; fi
  done
done
echo done
