set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_backward.py -m gpu -x -q -k "deterministic or bucket or exact" --timeout 200 --timeout-method thread > gpurun_out/pytest_order.log 2>&1 || { echo "pytest failed"; tail -20 gpurun_out/pytest_order.log; exit 1; }
tail -1 gpurun_out/pytest_order.log
bash tools/ab.sh "--mode train" "" "--tune wgrad_after_dgrad=1"
