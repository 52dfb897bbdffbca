set -e
export TMPDIR=/tmp
O=gpurun_out/r2s3_check
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -c 600 $O/bench.log
