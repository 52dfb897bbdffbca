set -e
export TMPDIR=/tmp
O=gpurun_out/v13
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_precision.py tests/test_gpu_forward.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/ab.sh "" "X=0" "HKP_LIB_AB=tools/bin/libhulkkp_base.so"
bash tools/ab.sh "--backbone resnet50 --keypoints 8 --batch 128 --precision f16" "X=0" "HKP_LIB_AB=tools/bin/libhulkkp_base.so"
