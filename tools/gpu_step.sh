set -o pipefail
export TMPDIR=/tmp
bash tools/ab.sh "--mode train" "" "--tune dgrad_overlap_tile=0" "--tune dgrad_overlap_tile=3" "--tune overlap_wgrad=0"
