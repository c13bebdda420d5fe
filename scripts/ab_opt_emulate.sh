#!/bin/bash
# Interleaved A/B of one ctx option in the per-shard emulation:
#   scripts/ab_opt_emulate.sh OPT "VAL1 VAL2 ..." [REPS] [WORLDS] [DELIVERY]
set -e
OPT=$1; VALS=$2; REPS=${3:-3}; WORLDS=${4:-8}; DELIVERY=${5:-host-direct}
for rep in $(seq "$REPS"); do
  for v in $VALS; do
    echo "## rep $rep cfg $OPT=$v"
    python -u scripts/multi_emulate.py --worlds "$WORLDS" --delivery "$DELIVERY" --opt "$OPT=$v"
  done
done
