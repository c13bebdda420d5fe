#!/bin/bash
# Time-based PC sampling (rocprofv3 host trap) of the bench's frame kernels,
# from a build with line tables (scripts/build_variant.sh g -gline-tables-only:
# the same code, plus .loc info), one launch at a time:
#   bash scripts/pc_sample.sh OUTDIR [bench args...]
set -u
OUT=$1; shift
mkdir -p "$OUT"
MIRT_LIB=${MIRT_LIB:-ab/libmirt_g.so} timeout -k 10 -s KILL 180 rocprofv3 --pc-sampling-beta-enabled \
    --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 1 \
    --output-format csv -d "$OUT" -o run -- python3 bench.py --no-cpu --no-host --pipeline 1 --steps 5 --warmup 2 "$@"
