#!/bin/bash
# Counter probe of the render kernel: SQ instruction mix / stalls per schedule.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmc}
mkdir -p "$OUT"
timeout -k 10 120 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
timeout -k 10 300 python3 scripts/profile_kernel.py --counts > "$OUT/counts.jsonl" 2>&1 || exit $?
for cfg in "0 1 1" "0 1 5" "2 1 5" "1 1 5"; do
  set -- $cfg
  tag=t$1_f$2_d$3
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY \
      -T --output-format csv -d "$OUT/$tag.a" -o run -- python3 scripts/profile_kernel.py --trav $1 --fast $2 --depth $3 --frames 2 > "$OUT/$tag.a.log" 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INST_CYCLES_SMEM GRBM_GUI_ACTIVE \
      -T --output-format csv -d "$OUT/$tag.b" -o run -- python3 scripts/profile_kernel.py --trav $1 --fast $2 --depth $3 --frames 2 > "$OUT/$tag.b.log" 2>&1 || exit $?
done
echo done
