#!/bin/bash
# GPU parity (pytest -m gpu on the in-tree libmirt.so) then scripts/ab_libs.py at 1080p/10k and 1080p/100k:
#   scripts/ab_round.sh <tag> ab/libmirt_base.so ab/libmirt_x.so
T=$1; shift
mkdir -p gpurun_out/$T && timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 && tail -n 2 gpurun_out/$T/pytest.log && timeout -k 10 300 python scripts/ab_libs.py "$@" --rounds 3 > gpurun_out/$T/ab_10k.log 2>&1 && timeout -k 10 300 python scripts/ab_libs.py "$@" --rounds 2 --workload 1080p_100k > gpurun_out/$T/ab_100k.log 2>&1 && grep BEST gpurun_out/$T/ab_*.log
