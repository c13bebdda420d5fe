#!/bin/bash
# Counter A/B of the frame kernels under option settings, one small counter
# set per rocprofv3 pass:
#   scripts/pmc_ab.sh <tag> <depth> "<name>:<opt=val>,<opt=val>" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/$1; DEPTH=$2; shift 2
mkdir -p "$OUT"
# extra counter sets: PMC_EXTRA="SET A COUNTERS;SET B COUNTERS"
SETS=(
 "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU"
 "SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_IFETCH GRBM_GUI_ACTIVE"
)
if [ -n "${PMC_EXTRA:-}" ]; then IFS=';' read -ra extra <<< "$PMC_EXTRA"; SETS+=("${extra[@]}"); fi
for cfg in "$@"; do
  name=${cfg%%:*}; opts=${cfg#*:}
  args=()
  IFS=, read -ra kv <<< "$opts"
  for o in "${kv[@]}"; do [ -n "$o" ] && args+=(--opt "$o"); done
  i=0
  for cs in "${SETS[@]}"; do
    i=$((i+1))
    timeout -k 10 90 rocprofv3 --pmc $cs --output-format csv -d "$OUT/t${name}_f1_d$DEPTH.$i" -o run -- \
        python3 scripts/profile_kernel.py --trav 5 --fast 1 --depth $DEPTH --frames 2 "${args[@]}" > "$OUT/$name.$i.log" 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "$name set $i rc=$rc"; grep -m3 -i "error\|not" "$OUT/$name.$i.log"; [ $rc -gt 1 ] && exit $rc; fi
  done
done
echo done
