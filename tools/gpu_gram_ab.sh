set -e
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/gram
timeout -k 10 300 python -u -m pytest tests/test_gpu_gram.py tests/test_gpu_precision.py tests/test_gpu_scale.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gram or c4 or r50" > gpurun_out/gram/pytest.log 2>&1 || { tail -30 gpurun_out/gram/pytest.log; exit 1; }
tail -1 gpurun_out/gram/pytest.log
for r in 1 2; do
timeout -k 10 120 python -u tools/gram_time.py --lib tools/ab_lib/libhulkkp_a.so
timeout -k 10 120 python -u tools/gram_time.py
done
bash tools/ab.sh "--backbone resnet50 --keypoints 8 --batch 128 --precision f16" "--lib tools/ab_lib/libhulkkp_a.so" ""
