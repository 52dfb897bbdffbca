mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_precision.py -x -q --timeout 200 --timeout-method thread > gpurun_out/prec.log 2>&1 || { tail -20 gpurun_out/prec.log; exit 1; }
bash tools/gpu_ab_bench.sh
