set -e
export TMPDIR=/tmp
O=gpurun_out/v5
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_precision.py tests/test_gpu_forward.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python -u -m pytest tests/test_gpu_precision.py -q -s -k "f16_forward_close" --timeout 120 --timeout-method thread 2>&1 | grep "fp16 R50"
timeout -k 10 200 python -u tools/x3_stamps.py c4_l4_c3 c4_l1_c3 c4_l4_c1
bash tools/ab.sh "--backbone resnet50 --keypoints 8 --batch 128 --precision f16" "X=0"
bash tools/ab.sh "" "X=0"
bash tools/pmc_passes.sh $O/pmc_infer "--steps 5 --no-extras" "conv_x3" > $O/pmc.log 2>&1
cat $O/pmc_infer/pmc_summary.txt
