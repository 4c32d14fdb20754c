#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
run() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-8} $OUT/$name.log; if [ $rc -ne 0 ]; then echo STOP; exit $rc; fi; }
TAILN=4 run r3_gemm_tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_prefill_gemm.py
for sch in ${SCHEDULES:-hybrid dp}; do
  TAILN=13 run r3_gemm_ab_$sch 400 python scripts/gpu/bench_prefill_gemm.py --m 512 1300 2600 --schedule $sch
  TAILN=13 run r3_gemm_ab_fp8_$sch 400 python scripts/gpu/bench_prefill_gemm.py --m 512 1300 2600 --fp8 --schedule $sch
done
