#!/bin/bash
# One GPU-box session (the one runner for every gpurun call): named steps,
# each under its own time limit, output in gpurun_out/<tag>/<step>.log. A
# fault / abort / timeout (rc not in {0,1}) ends the session: nothing more
# touches the GPU after it.
#
# usage: scripts/gpu_round.sh TAG STEP...
#   STEP is a preset below, or NAME=LIMIT=COMMAND (one argument, quoted), e.g.
#   scripts/gpu_round.sh r06b tests 'emu8=300=python scripts/multi_emulate.py --worlds 8'
#   presets: smoke tests multi bench bench_wl prof pmc
#   STRICT=1: stop at rc 1 too (a failed test or check)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r06}; shift || true
[ $# -eq 0 ] && set -- smoke tests bench prof pmc
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
step() {
    local name=$1 lim=$2; shift 2
    echo "== $name ($(date +%T))"
    timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -n 4 "$OUT/$name.log"
    if [ $rc -ne 0 ] && { [ $rc -ne 1 ] || [ "${STRICT:-0}" = 1 ]; }; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
for s in "$@"; do
  case $s in
    *=*=*) name=${s%%=*}; rest=${s#*=}; lim=${rest%%=*}; cmd=${rest#*=}
           step "$name" "$lim" bash -c "$cmd";;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()";;
    tests) step pytest_gpu 900 $PYT tests -m gpu;;
    multi) step pytest_multi 600 $PYT tests/test_multi.py -m gpu -s;;
    bench) step bench 600 python bench.py;;
    bench_wl) for wl in 1080p_100k 4k_10k 4k_1m_4spp; do step bench_$wl 600 python bench.py --workload $wl --no-cpu; done;;
    # one launch at a time (--pipeline 1): per-kernel durations as bench.py's serial measurement loop sees them
    prof)  step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --no-cpu --no-host --pipeline 1;;
    pmc)   step pmc_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 bench.py --no-cpu --no-host --steps 5 --warmup 1 --pipeline 1
           step pmc_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python3 bench.py --no-cpu --no-host --steps 5 --warmup 1 --pipeline 1;;
    *) echo "unknown step $s"; exit 2;;
  esac
done
echo "done"
