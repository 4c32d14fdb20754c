#!/bin/bash
# split-K routing in the engine: GEMM + engine tests, then prefill TTFT with / without it
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -q -x --timeout 120 --timeout-method thread -m gpu tests/test_prefill_gemm.py tests/test_engine.py > gpurun_out/sk2_tests.log 2>&1
rc=$?; tail -3 gpurun_out/sk2_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for pg in auto hipblaslt; do
    echo "== prefill_gemm=$pg"
    timeout -k 10 200 python scripts/gpu/prefill_bench.py --tokens 512,800,1024 --reps 7 --set prefill_gemm=$pg 2>&1 | grep prefill || exit 1
  done
done
