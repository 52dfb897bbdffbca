set -e
export TMPDIR=/tmp
O=gpurun_out/fin
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/ab.sh "" "X=0" "HKP_FIN_ONE_KERNEL=1"
bash tools/ab.sh "--backbone resnet50 --keypoints 8 --batch 128 --precision f16" "X=0" "HKP_FIN_ONE_KERNEL=1"
bash tools/ab.sh "--mode train" "X=0" "HKP_FIN_ONE_KERNEL=1"
