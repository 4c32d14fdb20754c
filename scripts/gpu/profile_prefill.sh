#!/bin/bash
# rocprofv3 kernel trace + stats of the prefill microbenchmark (no PMC counters).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_prefill
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
  python3 scripts/gpu/prefill_bench.py --tokens ${TOKENS:-2600} --reps ${REPS:-3} ${ARGS:-} \
  > gpurun_out/prof_prefill.log 2>&1
rc=$?
echo "rc=$rc"; cat gpurun_out/prof_prefill.log | grep prefill
python3 scripts/gpu/summarize_trace.py $OUT --window stream_read_kernel > gpurun_out/prof_prefill_summary.txt 2>&1
head -45 gpurun_out/prof_prefill_summary.txt
python3 scripts/gpu/trace_window.py $OUT sample_kernel 45 > gpurun_out/prof_prefill_window.txt 2>&1
find $OUT -name "*kernel_trace.csv" -delete
exit $rc
