#!/bin/bash
# Round 4: shading arithmetic -- successive RNG draws stepped instead of
# multiplied out (MIRT_DRAW_STEP): parity through the variant, then the A/B
# against the committed build. First: are gfx950's binary32 square roots
# correctly rounded (all 2^32 inputs against the binary64 root rounded)?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04ab
mkdir -p $OUT
timeout -k 10 60 ./scripts/sqrt_exhaustive > $OUT/sqrt_exhaustive.log 2>&1; cat $OUT/sqrt_exhaustive.log
timeout -k 10 600 env MIRT_LIB=ab/libmirt_step.so python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu_step.log 2>&1 || { tail -30 $OUT/pytest_gpu_step.log; exit 1; }
tail -1 $OUT/pytest_gpu_step.log
L="ab/libmirt_base.so ab/libmirt_step.so"
timeout -k 10 500 python scripts/ab_libs.py $L --rounds 3 --steps 20 > $OUT/ab_10k.log 2>&1 || exit 1
timeout -k 10 500 python scripts/ab_libs.py $L --rounds 2 --steps 20 --workload 1080p_100k > $OUT/ab_100k.log 2>&1 || exit 1
timeout -k 10 600 python scripts/ab_libs.py $L --rounds 1 --steps 20 --workload 4k_1m_4spp > $OUT/ab_4k1m.log 2>&1 || exit 1
grep BEST $OUT/ab_*.log
