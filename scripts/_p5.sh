set -o pipefail
mkdir -p gpurun_out/p5
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/p5/pytest.log 2>&1; rc=$?; tail -5 gpurun_out/p5/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python scripts/tail_fit.py &&
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/p5/bench.log 2>&1; tail -1 gpurun_out/p5/bench.log | cut -c1-700
