#!/bin/bash
# Round 4: normalize3's square root as the binary32 sqrtf (correctly rounded
# on gfx950: all 2^32 inputs equal the binary64 root rounded, r04ab) instead
# of the binary64 root -- parity through the variant, then the A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04ac
mkdir -p $OUT
timeout -k 10 600 env MIRT_LIB=ab/libmirt_sq32.so python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu_sq32.log 2>&1 || { tail -30 $OUT/pytest_gpu_sq32.log; exit 1; }
tail -1 $OUT/pytest_gpu_sq32.log
L="ab/libmirt_base.so ab/libmirt_sq32.so"
timeout -k 10 500 python scripts/ab_libs.py $L --rounds 3 --steps 20 > $OUT/ab_10k.log 2>&1 || exit 1
timeout -k 10 500 python scripts/ab_libs.py $L --rounds 2 --steps 20 --workload 1080p_100k > $OUT/ab_100k.log 2>&1 || exit 1
grep BEST $OUT/ab_*.log
for lib in base sq32; do
  timeout -k 10 200 env MIRT_LIB=ab/libmirt_$lib.so python scripts/blocking_frame.py --bounce-blocks 0,1280,1024,768,512 > $OUT/blocking_$lib.log 2>&1 || exit 1
  echo "$lib $(tail -1 $OUT/blocking_$lib.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in d if k.startswith("pinned") and k.endswith("_ms") or k == "kernels_ms"}, d["frames_equal"])')"
done
