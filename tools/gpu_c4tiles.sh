# C4 tile-policy A/B on the final tree (plain-fp16 1x1 and kxk convs)
set -e
export TMPDIR=/tmp
bash tools/ab.sh "--backbone resnet50 --keypoints 8 --batch 128 --precision f16" "X=0" "HKP_F16_TILE_1X1=7" "HKP_F16_TILE_1X1=2" "HKP_F16_TILE_1X1=4" "HKP_F16_TILE_KXK=2" "HKP_F16_TILE_KXK=7"
