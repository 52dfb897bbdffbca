set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
timeout -k 10 400 python -u -m pytest tests/test_gpu_precision.py tests/test_gpu_gram.py tests/test_gpu_scale.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03/pytest_half.log 2>&1 || { echo "pytest failed"; grep -E "Error|error|assert|FAILED" gpurun_out/r03/pytest_half.log | head -30; tail -5 gpurun_out/r03/pytest_half.log; exit 1; }
tail -1 gpurun_out/r03/pytest_half.log
S=c4_l4_c1,c4_l4_c3,c4_l4_c2,c4_l3_c1,c4_l3_c3,c4_l3_c2,c4_l1_c3
timeout -k 10 300 python -u tools/conv_ab.py --tiles 0 --rounds 5 --shapes $S --lib tools/bin/libhulkkp_prev.so 2>&1 | grep tile | sed 's/^/prev /'
timeout -k 10 300 python -u tools/conv_ab.py --tiles 0 --rounds 5 --shapes $S 2>&1 | grep tile | sed 's/^/new  /'
C4="--backbone resnet50 --keypoints 8 --batch 128 --precision f16"
bash tools/ab.sh "$C4" "--lib tools/bin/libhulkkp_prev.so" ""
