#!/bin/bash
# Round 5, session al: the fuzzed-view soak on this round's build (512 views
# per scene generator against the oracle, byte for byte) and the whole-frame
# parity of every BASELINE config.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r05al
mkdir -p $OUT
MIRT_FUZZ_CASES=512 timeout -k 10 600 python -u -m pytest tests/test_gpu_fuzz.py -m gpu -x -v --timeout 500 --timeout-method thread > $OUT/fuzz512.log 2>&1 || { echo "fuzz failed"; tail -20 $OUT/fuzz512.log; exit 1; }
tail -1 $OUT/fuzz512.log
timeout -k 10 600 python -u -m pytest tests/test_full_frames.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/full_frames.log 2>&1 || { echo "full frames failed"; tail -20 $OUT/full_frames.log; exit 1; }
tail -1 $OUT/full_frames.log
