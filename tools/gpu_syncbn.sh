# SyncBN GPU tests (inference + training), then the full GPU suite and a train-mode bench line
set -e
export TMPDIR=/tmp
O=gpurun_out/syncbn2
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_syncbn.py -x -v -s --timeout 300 --timeout-method thread > $O/pytest_syncbn.log 2>&1 || { tail -40 $O/pytest_syncbn.log; exit 1; }
grep -E "passed|failed|rel err" $O/pytest_syncbn.log | tail -6
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u bench.py --mode train --no-extras --no-cpu-baseline > $O/bench_train.log 2>&1 || { tail -20 $O/bench_train.log; exit 1; }
tail -1 $O/bench_train.log | cut -c1-200
