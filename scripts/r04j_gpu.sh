#!/bin/bash
# Round 4: chain bookkeeping in LDS (MIRT_CHAIN_LDS) at 5 and 6 bounce waves
# per SIMD (6: 16-entry lane stacks so six workgroups' LDS fit the CU).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=r04j
mkdir -p gpurun_out/$T
L="ab/libmirt_base.so ab/libmirt_c5.so ab/libmirt_c6s16.so ab/libmirt_w6s16.so"
for lib in ab/libmirt_c5.so ab/libmirt_c6s16.so; do
  MIRT_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_full_frames.py -m gpu -x -q --timeout 120 --timeout-method thread -k "golden or full or shared or bounce or quad" > gpurun_out/$T/pytest_$(basename $lib .so).log 2>&1 || { tail -20 gpurun_out/$T/pytest_$(basename $lib .so).log; exit 1; }
  tail -n 1 gpurun_out/$T/pytest_$(basename $lib .so).log
done
timeout -k 10 400 python scripts/ab_libs.py $L --rounds 2 --steps 20 > gpurun_out/$T/ab_10k.log 2>&1 || exit 1
timeout -k 10 400 python scripts/ab_libs.py $L --rounds 2 --steps 20 --workload 1080p_100k > gpurun_out/$T/ab_100k.log 2>&1 || exit 1
grep BEST gpurun_out/$T/ab_*.log
export GPU_MAX_HW_QUEUES=16
S="python3 scripts/shard_times.py --pipeline 8 --steps 5 --copy --batch 4"
for c in "--worlds 1,8" "--worlds 8 --tail-grid 2" "--worlds 8 --tail-grid 3" "--worlds 8 --tail-grid 2 --blocks 512" "--worlds 8 --tail-grid 5" "--worlds 1,8 --tail-grid 2 --width 3840 --height 2160" "--worlds 1,8 --width 3840 --height 2160"; do
  timeout -k 10 200 $S $c > gpurun_out/$T/emu.log.tmp 2>&1 || { tail -3 gpurun_out/$T/emu.log.tmp; exit 1; }
  echo "## $c" >> gpurun_out/$T/emu.log; grep '^{' gpurun_out/$T/emu.log.tmp >> gpurun_out/$T/emu.log
done
rm -f gpurun_out/$T/emu.log.tmp
grep -h pred_job gpurun_out/$T/emu.log | python3 -c "import sys,json; [print(d['world'],d['tail_grid'],d['blocks'],d['size'],d['pred_job_mrays_s_no_gather']) for d in map(json.loads,sys.stdin)]"
