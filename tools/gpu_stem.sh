set -e
export TMPDIR=/tmp
O=gpurun_out/stem
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_forward.py tests/test_gpu_precision.py tests/test_gpu_backward.py tests/test_gpu_datapath.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/ab.sh "" "X=0" "HKP_LIB_AB=tools/bin/libhulkkp_base.so"
bash tools/ab.sh "--backbone resnet50 --keypoints 8 --batch 128 --precision f16" "X=0" "HKP_LIB_AB=tools/bin/libhulkkp_base.so"
