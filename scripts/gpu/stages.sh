#!/bin/bash
# Staged GPU-box runner: STAGES="a b c" runs each named stage under its own time limit and
# stops at the first failure (a GPU fault, abort or timeout ends the call - nothing else is
# started on the GPU after it).  Replaces the round-3 one-off r3_*.sh probes.
#
#   STAGES="bench prefill" bash scripts/gpu/stages.sh
#
# Stages:
#   tests      pytest -m gpu (PYTEST_ARGS: files; PYTEST_K: a -k expression)
#   smoke      __graft_entry__.smoke()
#   bench      bench.py --steps $STEPS --warmup 1 --verbose ($BENCH_ARGS)
#   http       bench.py --via http ($BENCH_ARGS)
#   prefill    scripts/gpu/prefill_bench.py --tokens $TOKENS --seqs $SEQS ($PF_ARGS)
#   profpf     rocprofv3 kernel trace of prefill_bench, windowed summary
#   profbench  rocprofv3 kernel trace of bench.py, windowed summary
#   gemm       scripts/gpu/bench_prefill_gemm.py $GEMM_ARGS
#   py         python $PY_ARGS (any probe script)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
TAG=${TAG:-r4}
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name"
  timeout -k 10 "$t" "$@" > "$OUT/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -"${TAILN:-4}" "$OUT/${TAG}_$name.log"
  if [ $rc -ne 0 ]; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
for s in ${STAGES:-bench}; do
  case $s in
    tests) TAILN=6 run tests "${TEST_TIMEOUT:-900}" python -u -m pytest -x -q --timeout 240 \
             --timeout-method thread -m gpu ${PYTEST_K:+-k "$PYTEST_K"} ${PYTEST_ARGS:-tests} ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 900 python bench.py --steps "${STEPS:-2}" --warmup 1 --verbose ${BENCH_ARGS:-} ;;
    http) run http 900 python bench.py --via http --steps "${STEPS:-2}" --warmup 1 --verbose ${BENCH_ARGS:-} ;;
    prefill) TAILN=12 run prefill 600 python scripts/gpu/prefill_bench.py --tokens "${TOKENS:-400}" \
               --seqs "${SEQS:-5}" --reps "${REPS:-5}" ${PF_ARGS:-} ;;
    profpf)
      D=$OUT/${TAG}_profpf; rm -rf "$D"; mkdir -p "$D"
      TAILN=2 run profpf 700 rocprofv3 --kernel-trace --stats --output-format csv -d "$D" -o run -- \
        python3 scripts/gpu/prefill_bench.py --tokens "${TOKENS:-400}" --seqs "${SEQS:-5}" \
        --reps "${REPS:-3}" ${PF_ARGS:-}
      python3 scripts/gpu/summarize_trace.py "$D" --window stream_read_kernel > "$OUT/${TAG}_profpf_summary.txt" 2>&1
      head -30 "$OUT/${TAG}_profpf_summary.txt"
      find "$D" -name "*kernel_trace.csv" -delete ;;
    profbench)
      D=$OUT/${TAG}_profbench; rm -rf "$D"; mkdir -p "$D"
      ATTA_WINDOW_MARKERS=1 TAILN=2 run profbench 900 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$D" -o run -- python3 bench.py --steps 1 --warmup 1 ${BENCH_ARGS:-}
      python3 scripts/gpu/summarize_trace.py "$D" --window stream_read_kernel > "$OUT/${TAG}_profbench_summary.txt" 2>&1
      head -30 "$OUT/${TAG}_profbench_summary.txt"
      find "$D" -name "*kernel_trace.csv" -delete ;;
    gemm) TAILN=40 run gemm 600 python scripts/gpu/bench_prefill_gemm.py ${GEMM_ARGS:-} ;;
    py) TAILN=40 run py "${PY_TIMEOUT:-600}" python ${PY_ARGS} ;;
    *) echo "unknown stage $s"; exit 2 ;;
  esac
done
