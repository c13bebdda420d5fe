#!/bin/bash
# Build libmirt.so of a git revision into ab/libmirt_NAME.so (an A/B base for
# scripts/ab_libs.py), from a temporary worktree; the in-tree build is untouched.
#   scripts/build_rev.sh REV NAME
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
REV=$1 NAME=$2
WT=/tmp/mirt_rev_$NAME
rm -rf "$WT"; git -C "$ROOT" worktree prune
git -C "$ROOT" worktree add -q --detach "$WT" "$REV"
make -s -C "$WT/cs201_sah-bvh_ray_tracer_amd/csrc" -j8
mkdir -p "$ROOT/ab"
cp "$WT/cs201_sah-bvh_ray_tracer_amd/libmirt.so" "$ROOT/ab/libmirt_$NAME.so"
git -C "$ROOT" worktree remove --force "$WT"
echo "ab/libmirt_$NAME.so ($(git -C "$ROOT" rev-parse --short "$REV"))"
