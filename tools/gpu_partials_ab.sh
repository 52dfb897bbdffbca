set -e
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/partials
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
S=c4_l1_c3,c4_l2_c1a,c4_l4_c1,c4_l4_c2,layer4,layer3,layer2
timeout -k 10 300 python -u tools/conv_ab.py --tiles 0 --shapes $S --rounds 5 --iters 5 --lib tools/ab_lib/libhulkkp_a.so > $O/conv_a.log 2>&1
timeout -k 10 300 python -u tools/conv_ab.py --tiles 0 --shapes $S --rounds 5 --iters 5 > $O/conv_b.log 2>&1
paste -d'\n' $O/conv_a.log $O/conv_b.log | grep tile
bash tools/ab.sh "" "--lib tools/ab_lib/libhulkkp_a.so" ""
bash tools/ab.sh "--backbone resnet50 --keypoints 8 --batch 128 --precision f16" "--lib tools/ab_lib/libhulkkp_a.so" ""
