set -e
export TMPDIR=/tmp
O=gpurun_out/wg2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_precision.py -x -q --timeout 120 --timeout-method thread -k "wgrad" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  echo "== new"; timeout -k 10 120 python -u tools/wg_time.py --shapes t4,t3
  echo "== base"; HKP_LIB_AB=tools/bin/libhulkkp_base.so timeout -k 10 120 python -u tools/wg_time.py --shapes t4,t3
done
bash tools/ab.sh "--mode train" "X=0" "HKP_LIB_AB=tools/bin/libhulkkp_base.so"
