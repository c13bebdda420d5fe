set -o pipefail
mkdir -p gpurun_out/p7
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/p7/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/p7/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 250 python scripts/sweep.py --option 8 --values 0,1 --depth 5 && timeout -k 10 100 python scripts/tail_fit.py
