#!/bin/bash
# Round-3 evidence A: prefill GEMM routing (auto) tests, headline bench bf16 / fp8, windowed
# prefill + bench rocprof summaries.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
run() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 $t "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-3} $OUT/$name.log; if [ $rc -ne 0 ]; then echo STOP; exit $rc; fi; }
STAGES=${STAGES:-"tests bench bench8 profpf profpf8 profbench"}
for s in $STAGES; do case $s in
  tests) TAILN=3 run r3a_tests 600 python -u -m pytest -q --timeout 240 --timeout-method thread -m gpu tests/test_prefill_gemm.py tests/test_engine.py -k "prefill_gemm or fp8" ;;
  bench) run r3a_bench_bf16 600 python bench.py --steps 3 --warmup 1 ;;
  bench8) run r3a_bench_fp8 600 python bench.py --steps 3 --warmup 1 --quantization fp8 ;;
  profpf) TOKENS=512,2600 REPS=3 timeout -k 10 700 bash scripts/gpu/profile_prefill.sh > $OUT/r3a_profpf.log 2>&1; echo "profpf rc=$?"; cp $OUT/prof_prefill_summary.txt $OUT/r3a_prof_prefill_bf16_summary.txt; grep prefill $OUT/prof_prefill.log; head -25 $OUT/r3a_prof_prefill_bf16_summary.txt ;;
  profpf8) TOKENS=512,2600 REPS=3 ARGS="--quantization fp8" timeout -k 10 700 bash scripts/gpu/profile_prefill.sh > $OUT/r3a_profpf8.log 2>&1; echo "profpf8 rc=$?"; cp $OUT/prof_prefill_summary.txt $OUT/r3a_prof_prefill_fp8_summary.txt; grep prefill $OUT/prof_prefill.log; head -25 $OUT/r3a_prof_prefill_fp8_summary.txt ;;
  profbench) PROF_NAME=r3a_profbench STEPS=1 WARMUP=1 timeout -k 10 900 bash scripts/gpu/profile_bench.sh > $OUT/r3a_profbench.log 2>&1; echo "profbench rc=$?"; head -30 $OUT/r3a_profbench_summary.txt ;;
esac; done
