#!/bin/bash
# Lanes x frames-per-launch sweep of the per-shard emulation (host-direct,
# the bench's bounce grid), two interleaved reps: scripts/sweep_lanes.sh
set -e
for rep in 1 2; do
  python -u scripts/multi_emulate.py --worlds 2 --delivery host-direct --rounds 3 --sweep 8:1:0,10:1:0,12:1:0,16:1:0,10:2:0
  python -u scripts/multi_emulate.py --worlds 4 --delivery host-direct --rounds 3 --sweep 8:2:0,10:2:0,12:2:0,7:3:0,6:3:0,5:4:0
  python -u scripts/multi_emulate.py --worlds 8 --delivery host-direct --rounds 3 --sweep 8:4:0,5:4:0,6:4:0,10:2:0,7:3:0
done
