set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
timeout -k 10 600 python -u -m pytest tests/test_gpu_precision.py tests/test_gpu_gram.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03/pytest_halo_v1.log 2>&1 || { echo "pytest failed"; grep -E "Error|error|assert|FAILED" gpurun_out/r03/pytest_halo_v1.log | head -20; tail -5 gpurun_out/r03/pytest_halo_v1.log; exit 1; }
tail -1 gpurun_out/r03/pytest_halo_v1.log
timeout -k 10 300 python -u tools/conv_ab.py --tiles 0,6 --rounds 5 --shapes layer1,c4_l1_c2 > gpurun_out/r03/conv_halo.log 2>&1 && cat gpurun_out/r03/conv_halo.log | grep tile
for v in "" "--mode train"; do
  timeout -k 10 300 python -u bench.py $v --no-extras --no-cpu-baseline > gpurun_out/r03/c2.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r03/c2.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r03/c2.log').read().strip().splitlines()[-1]); print('[$v] %.1f img/s %.2f ms  %s %.3f' % (d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac']))"
done
timeout -k 10 300 python -u bench.py --backbone resnet50 --keypoints 8 --batch 128 --precision f16 --no-extras --no-cpu-baseline > gpurun_out/r03/c4_ab.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r03/c4_ab.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r03/c4_ab.log').read().strip().splitlines()[-1]); print('C4 %.1f img/s %.2f ms  %s %.3f' % (d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac']))"
