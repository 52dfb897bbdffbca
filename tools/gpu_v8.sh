set -e
export TMPDIR=/tmp
O=gpurun_out/v8
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_precision.py tests/test_gpu_backward.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/ab.sh "--mode train" "X=0"
