set -o pipefail
mkdir -p gpurun_out/p6
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/p6/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/p6/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/p6/bench.log 2>&1; tail -1 gpurun_out/p6/bench.log | cut -c1-300
