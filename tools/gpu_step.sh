set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
timeout -k 10 600 python -u -m pytest tests/test_gpu_gram.py tests/test_gpu_scale.py -k "gram or fused or c4 or r50" -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r03/pytest_gram_v2.log 2>&1 || { echo "pytest failed"; grep -E "Error|error|assert" gpurun_out/r03/pytest_gram_v2.log | head -20; tail -5 gpurun_out/r03/pytest_gram_v2.log; exit 1; }
tail -1 gpurun_out/r03/pytest_gram_v2.log
for v in "" "--tune gram_bn=0" "" "--tune gram_bn=0"; do
  timeout -k 10 300 python -u bench.py --backbone resnet50 --keypoints 8 --batch 128 --precision f16 --no-extras --no-cpu-baseline $v > gpurun_out/r03/c4_ab.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r03/c4_ab.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r03/c4_ab.log').read().strip().splitlines()[-1]); print('C4 [$v] %.1f img/s %.2f ms  %s %.3f' % (d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac']))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03/prof_c4b -o run -- python3 bench.py --backbone resnet50 --keypoints 8 --batch 128 --precision f16 --no-extras --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/r03/prof_c4b.log 2>&1 || { echo "prof failed"; exit 1; }
