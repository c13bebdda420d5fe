#!/bin/bash
# Counter probe of the render kernel for given schedules:
#   scripts/pmc_probe.sh <tag> "<trav> <fast> <depth>" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
SETS=(
 "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU"
 "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD"
 "TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TAGRAM0_REQ_sum TCP_TCC_READ_REQ_sum SQ_INSTS_SALU SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_LEVEL_WAVES"
)
for cfg in "$@"; do
  set -- $cfg
  tag=t$1_f$2_d$3
  i=0
  for cs in "${SETS[@]}"; do
    i=$((i+1))
    timeout -k 10 300 rocprofv3 --pmc $cs --output-format csv -d "$OUT/$tag.$i" -o run -- \
        python3 scripts/profile_kernel.py --trav $1 --fast $2 --depth $3 --frames 2 > "$OUT/$tag.$i.log" 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "$tag set $i rc=$rc"; tail -3 "$OUT/$tag.$i.log"; [ $rc -gt 1 ] && exit $rc; fi
  done
done
echo done
