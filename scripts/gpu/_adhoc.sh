set -o pipefail
set -e
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_wide_gemm.py -x -q -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/r5_ks_tests.log 2>&1 || { tail -30 gpurun_out/r5_ks_tests.log; exit 1; }
tail -1 gpurun_out/r5_ks_tests.log
timeout -k 10 400 python -u scripts/gpu/bench_wide.py --graph --plans --proj o down --m 33 50 75 85 95 105 128 > gpurun_out/r5_ks_bench_wide.txt 2>&1
cat gpurun_out/r5_ks_bench_wide.txt | grep -v amdgpu
for i in 1 2; do for v in 0 1; do
ATTA_WIDE_KS=$v timeout -k 10 600 python -u bench.py --steps 3 --warmup 2 > gpurun_out/r5_ks${v}_$i.log 2>&1
python -c "import json; d=json.loads(open('gpurun_out/r5_ks${v}_$i.log').read().strip().splitlines()[-1]); print('KS $v', d['value'], d['p50_ttft_s'], d['ttft_by_phase'])"
done; done
