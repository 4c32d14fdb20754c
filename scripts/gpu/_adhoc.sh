set -o pipefail
set -e
export PYTHONUNBUFFERED=1
for w in 4 8; do
ATTA_ATTN128_WAVES=$w timeout -k 10 300 python -u -m pytest tests/test_engine.py -k fp8_engine_matches_fp32_oracle -m gpu -q -s -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/r5_fp8oracle_w$w.log 2>&1 || true
echo "waves $w"; grep -E "fp8 oracle|passed|failed" gpurun_out/r5_fp8oracle_w$w.log
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/r5_gpu_tier_final2.log 2>&1 || { tail -40 gpurun_out/r5_gpu_tier_final2.log; exit 1; }
tail -3 gpurun_out/r5_gpu_tier_final2.log
