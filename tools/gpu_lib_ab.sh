# A/B of tools/ab_lib/libhulkkp_a.so (A) against the in-tree build (B) on one box:
#   bash tools/gpu_lib_ab.sh TAG CONV_SHAPES "BENCH ARGS" ["BENCH ARGS" ...]
# GPU suite first (stops on a failure), conv_ab per build, then tools/ab.sh per bench workload.
set -e
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:?tag}
S=${2:?shapes}
shift 2
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u tools/conv_ab.py --tiles 0 --shapes $S --rounds 5 --iters 5 --lib tools/ab_lib/libhulkkp_a.so > $O/conv_a.log 2>&1
timeout -k 10 300 python -u tools/conv_ab.py --tiles 0 --shapes $S --rounds 5 --iters 5 > $O/conv_b.log 2>&1
paste -d'\n' $O/conv_a.log $O/conv_b.log | grep tile
for B in "$@"; do
  bash tools/ab.sh "$B" "--lib tools/ab_lib/libhulkkp_a.so" ""
done
