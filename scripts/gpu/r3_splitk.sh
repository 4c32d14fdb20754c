#!/bin/bash
# split-K schedule of the prefill GEMM: fp32-oracle tests, then the A/B at small M
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread -m gpu tests/test_prefill_gemm.py > gpurun_out/sk_tests.log 2>&1
rc=$?; tail -3 gpurun_out/sk_tests.log; [ $rc -eq 0 ] || exit $rc
for sch in ${SCHEDULES:-splitk}; do
  timeout -k 10 300 python scripts/gpu/bench_prefill_gemm.py --schedule $sch --m ${MS:-400 512 1024} ${ONLY:+--only $ONLY} > gpurun_out/sk_ab_$sch.txt 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/sk_ab_$sch.txt
done
