set -o pipefail
export TMPDIR=/tmp
C4="--backbone resnet50 --keypoints 8 --batch 128 --precision f16"
bash tools/ab.sh "$C4" "" "--tune f16_tile_1x1=6" "--tune f16_tile_1x1=4" "--tune f16_tile_kxk=4"
