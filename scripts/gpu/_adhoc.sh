set -o pipefail
set -e
export PYTHONUNBUFFERED=1
ATTA_W16_UNROLL=1 timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_preshuffle.py -m gpu -x -q -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/r5_u4_tests.log 2>&1 || { tail -30 gpurun_out/r5_u4_tests.log; exit 1; }
tail -1 gpurun_out/r5_u4_tests.log
for i in 1 2; do for v in 2 1; do
ATTA_W16_UNROLL=$v timeout -k 10 600 python -u bench.py --steps 3 --warmup 2 > gpurun_out/r5_u${v}_$i.log 2>&1
python -c "import json; d=json.loads(open('gpurun_out/r5_u${v}_$i.log').read().strip().splitlines()[-1]); print('w16 unroll $v', d['value'], d['p50_ttft_s'])"
done; done
