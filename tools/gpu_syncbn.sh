# SyncBN GPU tests, then the full GPU suite and a default bench line
set -e
export TMPDIR=/tmp
O=gpurun_out/syncbn
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_syncbn.py -x -v -s --timeout 300 --timeout-method thread > $O/pytest_syncbn.log 2>&1 || { tail -40 $O/pytest_syncbn.log; exit 1; }
grep -E "passed|failed|low_err" $O/pytest_syncbn.log | tail -5
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
