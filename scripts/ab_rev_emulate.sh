#!/bin/bash
# Interleaved A/B of two library builds (MIRT_LIB) in the per-shard emulation:
#   scripts/ab_rev_emulate.sh LIB_A LIB_B [REPS] [WORLDS] [DELIVERY]
set -e
A=$1; B=$2; REPS=${3:-3}; WORLDS=${4:-2,4,8}; DELIVERY=${5:-host-direct}
for rep in $(seq "$REPS"); do
  for lib in "$A" "$B"; do
    echo "## rep $rep cfg $(basename "$lib")"
    MIRT_LIB=$(readlink -f "$lib") python -u scripts/multi_emulate.py --worlds "$WORLDS" --delivery "$DELIVERY"
  done
done
