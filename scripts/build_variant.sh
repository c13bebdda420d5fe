#!/bin/bash
# Build libmirt.so variants for an A/B (scripts/ab_libs.py / ab_session.sh):
#   scripts/build_variant.sh NAME "-DMACRO=VALUE ..." [NAME2 "FLAGS2" ...]
# Each variant is compiled in its own object directory and copied to
# ab/libmirt_NAME.so; the in-tree library is left as it was.
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CSRC=$ROOT/cs201_sah-bvh_ray_tracer_amd/csrc
mkdir -p "$ROOT/ab"
while [ $# -ge 2 ]; do
    name=$1 flags=$2; shift 2
    obj=/tmp/mirt_variant_$name
    rm -rf "$obj"; mkdir -p "$obj"
    common="-O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function $flags"
    for f in host_scene bvh_build bvh_cache dropin; do
        /opt/rocm/bin/hipcc $common --offload-arch=gfx950 -c "$CSRC/$f.cpp" -o "$obj/$f.o" &
    done
    for f in render multi; do
        /opt/rocm/bin/hipcc $common --offload-arch=gfx950 -c "$CSRC/$f.hip" -o "$obj/$f.o" &
    done
    wait
    /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$ROOT/ab/libmirt_$name.so" "$obj"/*.o \
        -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
    echo "ab/libmirt_$name.so ($flags)"
done
