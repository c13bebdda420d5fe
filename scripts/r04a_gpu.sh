#!/bin/bash
# Round 4, first box session: the GPU suite (new mirt_multi + drop-in tests
# first), the smoke test, the gather probe and its counter passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04a
mkdir -p "$OUT"
step() {
    local name=$1 lim=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -n 3 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step pytest_new 300 python -u -m pytest tests/test_multi.py tests/test_c_dropin.py -m gpu -x -v --timeout 200 --timeout-method thread
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
step blocking 120 python scripts/blocking_frame.py
step bstats_10k 120 python scripts/bounce_stats.py --spheres 10000
step bstats_100k 180 python scripts/bounce_stats.py --spheres 100000
step td_probe 60 ./scripts/td_probe
step td_pmc_acc 60 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d "$OUT/td_pmc_acc" -o run -- ./scripts/td_probe
step td_pmc_busy 60 rocprofv3 --pmc TD_TD_BUSY_sum TA_TA_BUSY_sum GRBM_GUI_ACTIVE --output-format csv -d "$OUT/td_pmc_busy" -o run -- ./scripts/td_probe
echo done
