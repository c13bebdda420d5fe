#!/bin/bash
# Round 4: scalar-cache warming in the camera-packet walk (both inner
# children's PNodes requested once the current node's boxes are in, so the
# next step's node load hits the scalar cache) -- parity through the variant
# library, then the A/B against the committed build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04w
mkdir -p $OUT
timeout -k 10 600 env MIRT_LIB=ab/libmirt_warm.so python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu_warm.log 2>&1 || { tail -30 $OUT/pytest_gpu_warm.log; exit 1; }
tail -1 $OUT/pytest_gpu_warm.log
L="ab/libmirt_base.so ab/libmirt_warm.so"
timeout -k 10 400 python scripts/ab_libs.py $L --rounds 3 --steps 20 > $OUT/ab_10k.log 2>&1 || exit 1
timeout -k 10 400 python scripts/ab_libs.py $L --rounds 2 --steps 20 --workload 1080p_100k > $OUT/ab_100k.log 2>&1 || exit 1
timeout -k 10 600 python scripts/ab_libs.py $L --rounds 1 --steps 20 --workload 4k_1m_4spp > $OUT/ab_4k1m.log 2>&1 || exit 1
grep BEST $OUT/ab_*.log
